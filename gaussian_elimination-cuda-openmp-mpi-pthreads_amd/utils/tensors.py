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


_DEDICATED: dict[tuple[int, str], torch.cuda.ExternalStream] = {}
_DEDICATED_LOCK = __import__("threading").Lock()


def dedicated_stream(device: torch.device, role: str) -> torch.cuda.ExternalStream:
    """The process-lifetime stream of `role` on `device` ("side": the
    lookahead trailing-update stream of the distributed solvers, "comm": the
    stream RCCL collectives are issued on, parallel/comm.py).

    HIP maps streams onto GPU_MAX_HW_QUEUES (4) hardware queues per process
    and shares queues once they run out; a lookahead stream on the default
    stream's queue silently serialises behind it (the distributed 2048 solve
    took 16 instead of 8 ms, profiles/hw_queues_r4.txt), and a collective on
    the side stream's queue would wait behind the whole trailing update.  So
    each role's stream is created natively (gelim_gpu_stream_create_probed)
    and probed to run beside the default stream AND every other role's stream
    already made on the device; the roles together take 3 of the 4 queues.
    Not one of torch's pool streams: torch hands those out round-robin to
    any later torch.cuda.Stream() caller, which could put unrelated work in
    the lookahead stream.  Created once per (device, role) and never
    destroyed, so solvers made and dropped in a loop do not create streams."""
    import ctypes
    import warnings

    from .. import _native

    key = (device.index if device.index is not None else torch.cuda.current_device(), role)
    with _DEDICATED_LOCK:
        s = _DEDICATED.get(key)
        if s is not None:
            return s
        lib = _native.lib()
        others = [v.cuda_stream for (d, _), v in _DEDICATED.items() if d == key[0]]
        arr = (ctypes.c_void_p * max(1, len(others)))(*others)
        out = ctypes.c_void_p()
        before = side_stream_stats()
        with torch.cuda.device(key[0]):
            _native.check(lib.gelim_gpu_stream_create_probed(ctypes.byref(out), arr, len(others)),
                          "stream_create_probed")
        after = side_stream_stats()
        if after[1] - before[1] >= 8:  # every try shared a queue: the last one is kept
            warnings.warn(f"no {role} stream found running beside the default stream and {len(others)} other "
                          f"dedicated stream(s) on cuda:{key[0]}; the lookahead may serialise", RuntimeWarning)
        s = torch.cuda.ExternalStream(out.value, device=torch.device("cuda", key[0]))
        _DEDICATED[key] = s
        return s


def side_stream(device: torch.device) -> torch.cuda.ExternalStream:
    """The lookahead side stream of the distributed solvers (shared by every
    solver -- and every emulated rank -- of the process on `device`)."""
    return dedicated_stream(device, "side")


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
