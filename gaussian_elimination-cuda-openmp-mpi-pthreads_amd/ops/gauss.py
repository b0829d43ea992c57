"""Reference-semantics CPU elimination backends (SEQ / OMP / Pthreads V1-V3)
on torch CPU tensors — thin wrappers over `gelim_cpu_gauss`
(csrc/cpu/gauss_cpu.cpp)."""
from __future__ import annotations

import torch

from .. import _native
from ..utils.tensors import ptr, row_major_ld

CPU_BACKENDS = {
    "seq": _native.CPU_SEQ,
    "omp": _native.CPU_OMP,
    "pthreads-v1": _native.CPU_PTH_V1,
    "pthreads-v2": _native.CPU_PTH_V2,
    "pthreads-v3": _native.CPU_PTH_V3,
}


def cpu_max_threads() -> int:
    return int(_native.lib().gelim_cpu_max_threads())


def cpu_gauss_(A: torch.Tensor, b: torch.Tensor, backend: str = "seq", pivot: str = "partial",
               threads: int = 0, affinity: bool = True) -> None:
    """Forward elimination in place: A -> unit upper triangle (zeros below),
    b transformed (reference computeGauss)."""
    if A.device.type != "cpu" or A.dtype != torch.float64 or b.dtype != torch.float64:
        raise TypeError("cpu_gauss_ needs float64 CPU tensors")
    if not b.is_contiguous():
        raise ValueError("b must be contiguous")
    n = A.shape[0]
    code = CPU_BACKENDS[backend]
    pv = _native.PIVOT_PARTIAL if pivot == "partial" else _native.PIVOT_ZERO
    _native.check(_native.lib().gelim_cpu_gauss(ptr(A), row_major_ld(A), ptr(b), n, pv, code, threads,
                                                int(affinity)), f"cpu_gauss[{backend}]")


def cpu_backsub_unit(U: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    n = U.shape[0]
    x = torch.empty(n, dtype=torch.float64)
    bc = b.contiguous()
    _native.lib().gelim_cpu_backsub_unit(ptr(U), row_major_ld(U), ptr(bc), ptr(x), n)
    return x


def error_metric(x: torch.Tensor) -> float:
    """max_i |x_i - (i+1)| / (i+1)  (gauss_external_input.c:308-315)."""
    xc = x.detach().to("cpu", torch.float64).contiguous()
    return float(_native.lib().gelim_error_metric(ptr(xc), xc.numel()))
