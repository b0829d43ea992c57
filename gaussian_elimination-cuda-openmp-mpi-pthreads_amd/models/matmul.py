"""MatMul — the framework's fp32 matrix-multiply "model" with the reference's
timing semantics (CUDA_and_OpenMP/Version-2/cuda_matmul.cu:135-165):

  end_to_end : device malloc + H2D(A, B) + kernel + D2H(C) + free
  kernel     : the kernel alone (HIP events)

Host inputs are pinned so the copies run at link speed; allocation of the
host arrays is outside the timer, as in the reference.
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
