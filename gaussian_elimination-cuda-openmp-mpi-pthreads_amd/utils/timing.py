"""Timers: reference-style wall clock (gettimeofday, P1i:278-290) and
device-side HIP event timing for kernel-only numbers."""
from __future__ import annotations

import time

import torch


def wall() -> float:
    return time.perf_counter()


class DeviceTimer:
    """Brackets a region with HIP events on the current stream; `.elapsed_s`
    synchronises on the end event."""

    def __init__(self, device: torch.device | None = None):
        self.device = device
        self.start = torch.cuda.Event(enable_timing=True)
        self.end = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.start.record()
        return self

    def __exit__(self, *exc):
        self.end.record()
        return False

    @property
    def elapsed_s(self) -> float:
        self.end.synchronize()
        return self.start.elapsed_time(self.end) * 1e-3
