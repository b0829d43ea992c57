"""System initialisers (host or device), all native.

Every initialiser returns augmented storage (n, ld) with ld >= n+1 whose
column n holds b, the layout the GPU solvers eliminate in place.
  synthetic : A[i][j] = 2 min(i+1,j+1), b[i] = i   (P1i:59-69)
  random    : A ~ U[-1,1) (counter hash, identical on host and device),
              b = A (1..n) so the exact solution is x_i = i+1
  external  : a `.dat` / fixture matrix, b = A (1..n) in the reference order
"""
from __future__ import annotations

import torch

from .. import _native
from ..utils.tensors import empty_augmented, ptr, stream_handle


def synthetic_system(n: int, device="cpu", dtype=torch.float64) -> torch.Tensor:
    device = torch.device(device)
    aug = empty_augmented(n, dtype, device)
    ld = aug.stride(0)
    lib = _native.lib()
    if device.type == "cuda":
        fn = lib.gelim_gpu_init_synthetic if dtype == torch.float64 else lib.gelim_gpu_init_synthetic_f32
        _native.check(fn(ptr(aug), ld, n, stream_handle(device)), "init_synthetic")
        return aug
    host = torch.zeros((n, ld), dtype=torch.float64)
    b = torch.empty(n, dtype=torch.float64)
    lib.gelim_init_synthetic_f64(ptr(host), ld, ptr(b), n)
    host[:, n] = b
    return host.to(dtype)


def random_system(n: int, seed: int = 0, device="cpu") -> torch.Tensor:
    device = torch.device(device)
    aug = empty_augmented(n, torch.float64, device)
    ld = aug.stride(0)
    lib = _native.lib()
    if device.type == "cuda":
        s = stream_handle(device)
        _native.check(lib.gelim_gpu_init_random(ptr(aug), ld, n, seed & (2**64 - 1), s), "init_random")
        _native.check(lib.gelim_gpu_init_rhs(ptr(aug), ld, n, s), "init_rhs")
        return aug
    lib.gelim_init_random_f64(ptr(aug), ld, n, seed & (2**64 - 1))
    r = torch.empty(n, dtype=torch.float64)
    lib.gelim_init_rhs_f64(ptr(aug), ld, ptr(r), n)
    aug[:, n] = r
    return aug


def augment_with_rhs(A: torch.Tensor) -> torch.Tensor:
    """[A | A (1..n)] with the RHS computed on the host in the reference's
    summation order (gauss_external_input.c:90-108)."""
    A = A.to("cpu", torch.float64)
    n = A.shape[0]
    aug = empty_augmented(n)
    aug[:, :n] = A[:, :n]
    r = torch.empty(n, dtype=torch.float64)
    _native.lib().gelim_init_rhs_f64(ptr(aug), aug.stride(0), ptr(r), n)
    aug[:, n] = r
    return aug
