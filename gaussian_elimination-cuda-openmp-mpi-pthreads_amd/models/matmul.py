"""MatMul — the framework's fp32 matrix-multiply "model" with the reference's
timing semantics (CUDA_and_OpenMP/Version-2/cuda_matmul.cu:135-165):

  end_to_end : device malloc + H2D(A, B) + kernel + D2H(C) + free
  kernel     : the kernel alone (HIP events)

Host inputs are pinned so the copies run at link speed; allocation of the
host arrays is outside the timer, as in the reference.

`run_pipelined` keeps the same timer scope but overlaps the transfers with
the GEMM: B goes up first, then A in row chunks on an H2D stream; each
chunk's C rows are multiplied on the compute stream as soon as the chunk has
landed and copied back on a D2H stream (PCIe is full duplex, so C's return
runs under A's upload).  The reference's three blocking copies
(cuda_matmul.cu:147-157) serialise ~50 MB of traffic behind one kernel.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops import matmul as mm
from ..utils.timing import DeviceTimer, wall


@dataclass
class MatMulTiming:
    end_to_end_s: float
    kernel_s: float
    n: int
    kernel: str

    @property
    def kernel_tflops(self) -> float:
        return 2.0 * self.n ** 3 / self.kernel_s * 1e-12


class MatMul:
    def __init__(self, kernel: str = "mfma", device="cuda"):
        if kernel not in mm.KERNELS:
            raise ValueError(f"kernel must be one of {tuple(mm.KERNELS)}")
        self.kernel = kernel
        self.device = torch.device(device)

    def __call__(self, A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
        return mm.matmul(A, B, self.kernel)

    def run_reference_style(self, A_host: torch.Tensor, B_host: torch.Tensor,
                            C_host: torch.Tensor) -> MatMulTiming:
        """One end-to-end GPU multiply with the reference's timer scope."""
        n = A_host.shape[0]
        torch.cuda.synchronize(self.device)
        t0 = wall()
        dA = A_host.to(self.device, non_blocking=False)
        dB = B_host.to(self.device, non_blocking=False)
        with DeviceTimer(self.device) as kt:
            dC = mm.matmul(dA, dB, self.kernel)
        C_host.copy_(dC)
        del dA, dB, dC
        torch.cuda.synchronize(self.device)
        e2e = wall() - t0
        return MatMulTiming(e2e, kt.elapsed_s, n, self.kernel)

    def run_pipelined(self, A_host: torch.Tensor, B_host: torch.Tensor, C_host: torch.Tensor,
                      chunks: int = 2) -> MatMulTiming:
        """End-to-end multiply (same timer scope as run_reference_style) with
        chunked H2D / GEMM / D2H overlap on three streams.  kernel_s is the
        sum of the per-chunk GEMM times.  Measured at 2048^2
        (profiles/matmul2048_pipeline_sweep.txt): 2 chunks 1.07 ms vs 1.17 ms
        serial; every extra chunk costs ~0.13 ms of per-copy overhead, so
        the default is 2."""
        n, dev = A_host.shape[0], self.device
        if not (A_host.is_pinned() and B_host.is_pinned() and C_host.is_pinned()):
            raise ValueError("run_pipelined needs pinned host tensors")
        bounds = [(n * c // chunks, n * (c + 1) // chunks) for c in range(chunks)]
        bounds = [(r0, r1) for r0, r1 in bounds if r1 > r0]
        cur = torch.cuda.current_stream(dev)
        if not hasattr(self, "_streams"):  # created once: stream creation is ~100 us
            self._streams = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
            self._events = []
        up, down = self._streams
        while len(self._events) < len(bounds):
            self._events.append((torch.cuda.Event(), torch.cuda.Event(enable_timing=True),
                                 torch.cuda.Event(enable_timing=True)))
        ev = self._events[:len(bounds)]
        torch.cuda.synchronize(dev)
        t0 = wall()
        dA = torch.empty_like(A_host, device=dev)
        dB = torch.empty_like(B_host, device=dev)
        dC = torch.empty((n, B_host.shape[1]), dtype=torch.float32, device=dev)
        with torch.cuda.stream(up):
            dB.copy_(B_host, non_blocking=True)
            for (r0, r1), (landed, _, _) in zip(bounds, ev):
                dA[r0:r1].copy_(A_host[r0:r1], non_blocking=True)
                landed.record(up)
        for (r0, r1), (landed, k0, k1) in zip(bounds, ev):
            cur.wait_event(landed)
            k0.record(cur)
            mm.matmul(dA[r0:r1], dB, self.kernel, out=dC[r0:r1])
            k1.record(cur)
            down.wait_event(k1)
            with torch.cuda.stream(down):
                C_host[r0:r1].copy_(dC[r0:r1], non_blocking=True)
        for t in (dA, dB, dC):
            t.record_stream(up)
            t.record_stream(down)
        del dA, dB, dC
        torch.cuda.synchronize(dev)
        e2e = wall() - t0
        ker = sum(k0.elapsed_time(k1) for _, k0, k1 in ev) * 1e-3
        return MatMulTiming(e2e, ker, n, self.kernel)
