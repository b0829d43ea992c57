"""Blocked-LU building blocks on torch tensors (row-major views).

Each op dispatches on the tensor's device to the native library: HIP kernels
(`csrc/hip/lu_*.hip`) for CUDA tensors, the C++ versions
(`csrc/cpu/gauss_cpu.cpp`) for CPU tensors — both native, no Python math.
Views may be sub-blocks of a larger row-major matrix (stride(1) == 1); the
leading dimension is taken from stride(0).

These are the steps of the blocked form of the reference's elimination loop
(OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182):
  panel_factor : pivot search + row swap + multipliers for w columns
  swap_trsm    : apply those w interchanges to other columns, U12 = L11^-1 A12
  gemm_update  : A22 -= L21 @ U12  (fp64 MFMA on the GPU)
  backsub      : U x = y
"""
from __future__ import annotations

import torch

from .. import _native
from ..utils.tensors import is_gpu, ptr, row_major_ld, stream_handle

PIVOT = {"zero": _native.PIVOT_ZERO, "partial": _native.PIVOT_PARTIAL}


def _pivot_code(pivot) -> int:
    return PIVOT[pivot] if isinstance(pivot, str) else int(pivot)


def _f64(*ts):
    for t in ts:
        if t.dtype != torch.float64:
            raise TypeError(f"expected float64, got {t.dtype}")


def panel_factor(P: torch.Tensor, piv: torch.Tensor, info: torch.Tensor, row0: int = 0,
                 pivot="partial") -> None:
    """Factor the m x w panel view P in place (L unit-lower below the diagonal,
    U on/above it); piv[j] (int32, length >= w) receives the local row swapped
    into position j; info (int32 scalar tensor) gets row0+j+1 at the first
    zero pivot if it was 0."""
    _f64(P)
    m, w = P.shape
    ld = row_major_ld(P)
    lib = _native.lib()
    if is_gpu(P):
        _native.check(lib.gelim_gpu_panel_factor(ptr(P), ld, m, w, row0, _pivot_code(pivot), ptr(piv),
                                                 ptr(info), stream_handle(P.device)), "panel_factor")
    else:
        _native.check(lib.gelim_cpu_panel_factor(ptr(P), ld, m, w, row0, _pivot_code(pivot), ptr(piv),
                                                 ptr(info)), "panel_factor")


def panel_max_rows(w: int) -> int:
    return int(_native.lib().gelim_gpu_panel_max_rows(w))


def swap_trsm(Cm: torch.Tensor, L: torch.Tensor, piv: torch.Tensor) -> None:
    """Cm: (nrows x ncols) view whose row 0 is the panel's first row.  Apply
    the w sequential interchanges j <-> piv[j], then Cm[:w] = L11^-1 Cm[:w]
    with L11 the unit-lower part of L[:w,:w]."""
    _f64(Cm, L)
    nrows, ncols = Cm.shape
    w = L.shape[1]
    if ncols == 0:
        return
    lib = _native.lib()
    if is_gpu(Cm):
        _native.check(lib.gelim_gpu_swap_trsm(ptr(Cm), row_major_ld(Cm), ncols, ptr(L), row_major_ld(L), w,
                                              ptr(piv), nrows, stream_handle(Cm.device)), "swap_trsm")
    else:
        _native.check(lib.gelim_cpu_swap_trsm(ptr(Cm), row_major_ld(Cm), ncols, ptr(L), row_major_ld(L), w,
                                              ptr(piv), 0, nrows), "swap_trsm")


def gemm_update(Cm: torch.Tensor, L: torch.Tensor, U: torch.Tensor) -> None:
    """Cm -= L @ U (fp64).  GPU: v_mfma_f64_16x16x4_f64 kernel."""
    _f64(Cm, L, U)
    M, N = Cm.shape
    K = L.shape[1]
    if M == 0 or N == 0 or K == 0:
        return
    if L.shape[0] != M or U.shape != (K, N):
        raise ValueError(f"gemm_update shapes: C{tuple(Cm.shape)} L{tuple(L.shape)} U{tuple(U.shape)}")
    lib = _native.lib()
    args = (ptr(Cm), row_major_ld(Cm), ptr(L), row_major_ld(L), ptr(U), row_major_ld(U), M, N, K)
    if is_gpu(Cm):
        _native.check(lib.gelim_gpu_gemm_update(*args, stream_handle(Cm.device)), "gemm_update")
    else:
        _native.check(lib.gelim_cpu_gemm_update(*args), "gemm_update")


def backsub(U: torch.Tensor, y: torch.Tensor, unit: bool = False, bnorm: torch.Tensor | None = None
            ) -> torch.Tensor:
    """Solve U x = y (U upper triangular n x n view, y a length-n vector view
    of any stride).  Returns x (float64, same device)."""
    _f64(U)
    n = U.shape[0]
    x = torch.empty(n, dtype=torch.float64, device=U.device)
    if is_gpu(U):
        _native.check(_native.lib().gelim_gpu_backsub(ptr(U), row_major_ld(U), ptr(y), y.stride(0), ptr(x),
                                                      ptr(bnorm), n, int(unit), stream_handle(U.device)),
                      "backsub")
        return x
    Uc = U.contiguous()
    if unit:
        yc = y.contiguous()
        _native.lib().gelim_cpu_backsub_unit(ptr(Uc), row_major_ld(Uc), ptr(yc), ptr(x), n)
        if bnorm is not None:
            bnorm.copy_(yc)
        return x
    # non-unit: scale rows by the diagonal, then the unit solve (same math)
    d = torch.diagonal(Uc).clone()
    Us = Uc / d[:, None]
    ys = (y / d).contiguous()
    if bnorm is not None:
        bnorm.copy_(ys)
    _native.lib().gelim_cpu_backsub_unit(ptr(Us), row_major_ld(Us), ptr(ys), ptr(x), n)
    return x
