"""Timers: reference-style wall clock (gettimeofday, P1i:278-290) and
device-side HIP event timing for kernel-only numbers."""
from __future__ import annotations

import statistics
import time
from dataclasses import dataclass, field

import torch


def wall() -> float:
    return time.perf_counter()


@dataclass
class Stats:
    samples: list[float] = field(default_factory=list)

    def add(self, v: float) -> None:
        self.samples.append(v)

    @property
    def median(self) -> float:
        return statistics.median(self.samples) if self.samples else float("nan")

    @property
    def minimum(self) -> float:
        return min(self.samples) if self.samples else float("nan")

    @property
    def mean(self) -> float:
        return statistics.fmean(self.samples) if self.samples else float("nan")

    def as_dict(self) -> dict:
        return {"median": self.median, "min": self.minimum, "mean": self.mean, "n": len(self.samples)}


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


class WallTimer:
    """Wall-clock region; with `sync=True` the current CUDA stream is
    synchronised on entry and exit (reference semantics: end-to-end)."""

    def __init__(self, sync: bool = False):
        self.sync = sync
        self.elapsed_s = 0.0

    def __enter__(self):
        if self.sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        self._t0 = wall()
        return self

    def __exit__(self, *exc):
        if self.sync and torch.cuda.is_available():
            torch.cuda.synchronize()
        self.elapsed_s = wall() - self._t0
        return False
