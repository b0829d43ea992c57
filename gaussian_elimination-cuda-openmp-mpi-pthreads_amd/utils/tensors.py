"""Tensor plumbing between torch and the native library: raw pointers,
leading dimensions and the HIP stream handle of the current torch stream."""
from __future__ import annotations

import torch


def ptr(t: torch.Tensor | None) -> int | None:
    """Raw data pointer (None for None)."""
    return None if t is None else t.data_ptr()


def row_major_ld(t: torch.Tensor) -> int:
    """Leading dimension of a row-major 2-D view (unit column stride)."""
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError(f"expected a row-major 2-D view with unit column stride, got strides {t.stride()}")
    return t.stride(0) if t.size(0) > 1 else max(t.stride(0), t.size(1))


def stream_handle(device: torch.device | None = None) -> int | None:
    """hipStream_t of torch's current stream on `device` (None on CPU)."""
    if device is not None and device.type != "cuda":
        return None
    return torch.cuda.current_stream(device).cuda_stream


def is_gpu(t: torch.Tensor) -> bool:
    return t.device.type == "cuda"


def padded_ld(ncols: int, elem_bytes: int = 8, align_bytes: int = 64) -> int:
    """Row pitch (elements) rounded so every row starts 64-byte aligned."""
    a = align_bytes // elem_bytes
    return (ncols + a - 1) // a * a


def empty_augmented(n: int, dtype=torch.float64, device="cpu") -> torch.Tensor:
    """Storage for an augmented system [A | b]: shape (n, ld) with ld >= n+1;
    the logical system is the view [:, :n+1]."""
    ld = padded_ld(n + 1, torch.empty((), dtype=dtype).element_size())
    return torch.zeros((n, ld), dtype=dtype, device=device)
