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


def side_stream(device: torch.device) -> torch.cuda.Stream:
    """A torch stream that runs BESIDE the default stream.  HIP shares
    hardware queues between streams once a process has created
    GPU_MAX_HW_QUEUES of them, and a lookahead stream on the default
    stream's queue silently serialises behind it (the distributed 2048 solve
    took 16 instead of 8 ms, profiles/hw_queues_r4.txt).  So torch's pool
    streams are probed (runtime.hip gelim_gpu_stream_probe: a bounded wait on
    the default stream for a flag the candidate sets) and the first one that
    runs concurrently is returned -- a pool stream, so its lifetime is
    torch's."""
    from .. import _native

    lib = _native.lib()
    s = None
    with torch.cuda.device(device):
        for _ in range(33):  # torch's pool holds 32 streams per priority
            s = torch.cuda.Stream(device)
            rc = int(lib.gelim_gpu_stream_probe(s.cuda_stream))
            if rc < 0:
                _native.check(rc, "stream_probe")
            if rc == 1:
                break
    return s


def side_stream_stats() -> tuple[int, int]:
    """(streams probed, streams found sharing the default stream's hardware
    queue) in this process."""
    from .. import _native

    import ctypes

    out = (ctypes.c_int32 * 2)()
    _native.lib().gelim_gpu_side_stream_stats(out)
    return int(out[0]), int(out[1])


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
