"""fp32 matrix multiply C = A @ B.

GPU kernels (csrc/hip/gemm_f32.hip):
  "mfma"       LDS-tiled v_mfma_f32_32x32x2_f32 GEMM (default)
  "naive-row"  K1 parity: one workgroup per output row (cuda_matmul.cu V1)
  "naive-elem" K2 parity: one thread per output element (cuda_matmul.cu V2)
CPU: the reference's own i-j-k loops (sequential or OpenMP), the speedup
denominator of the 578x headline.
"""
from __future__ import annotations

import torch

from .. import _native
from ..utils.tensors import ptr, stream_handle

KERNELS = {"naive-row": _native.MM_NAIVE_ROW, "naive-elem": _native.MM_NAIVE_ELEM, "mfma": _native.MM_MFMA}


def matmul(A: torch.Tensor, B: torch.Tensor, kernel: str = "mfma", out: torch.Tensor | None = None
           ) -> torch.Tensor:
    if A.dtype != torch.float32 or B.dtype != torch.float32:
        raise TypeError("matmul is fp32")
    if A.device.type != "cuda" or B.device != A.device:
        raise ValueError("GPU matmul needs CUDA tensors on one device; use cpu_matmul for the host loops")
    A = A.contiguous()
    B = B.contiguous()
    M, K = A.shape
    K2, N = B.shape
    if K != K2:
        raise ValueError(f"shape mismatch {tuple(A.shape)} @ {tuple(B.shape)}")
    C = out if out is not None else torch.empty((M, N), dtype=torch.float32, device=A.device)
    if not C.is_contiguous() or C.shape != (M, N):
        raise ValueError("out must be a contiguous (M, N) tensor")
    _native.check(_native.lib().gelim_gpu_matmul_f32(ptr(A), ptr(B), ptr(C), M, N, K, KERNELS[kernel],
                                                     stream_handle(A.device)), f"matmul[{kernel}]")
    return C


def cpu_matmul(A: torch.Tensor, B: torch.Tensor, omp: bool = False, threads: int = 0) -> torch.Tensor:
    """The reference's square i-j-k loop (cuda_matmul.cu:28-57)."""
    n = A.shape[0]
    if A.shape != (n, n) or B.shape != (n, n):
        raise ValueError("reference CPU matmul is square")
    A = A.contiguous().float()
    B = B.contiguous().float()
    C = torch.empty((n, n), dtype=torch.float32)
    _native.lib().gelim_cpu_matmul_f32(ptr(A), ptr(B), ptr(C), n, int(omp), threads)
    return C


def reference_inputs(n: int) -> tuple[torch.Tensor, torch.Tensor]:
    """A[idx] = idx+1, B[idx] = 1/(idx+1) (cuda_matmul.cu:121-132)."""
    A = torch.empty((n, n), dtype=torch.float32)
    B = torch.empty((n, n), dtype=torch.float32)
    _native.lib().gelim_init_matmul_f32(ptr(A), ptr(B), n)
    return A, B
