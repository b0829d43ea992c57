"""Vendor-library reference point: torch.linalg.solve (rocSOLVER getrf/getrs)
fp64 wall time per solve on one MI355X, for n in argv (default 2048 4096
8192).  Only a comparison number for profiles/ — never a code path.
"""
import sys
import time

import torch


def main() -> None:
    ns = [int(a) for a in sys.argv[1:]] or [2048, 4096, 8192]
    dev = torch.device("cuda:0")
    for n in ns:
        g = torch.Generator(device=dev).manual_seed(n)
        a = torch.rand(n, n, device=dev, dtype=torch.float64, generator=g) * 2 - 1
        x0 = torch.arange(1, n + 1, device=dev, dtype=torch.float64)
        b = a @ x0
        for _ in range(2):
            torch.linalg.solve(a, b)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            x = torch.linalg.solve(a, b)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        err = ((x - x0).abs() / x0.abs()).max().item()
        print(f"torch.linalg.solve fp64 n={n}: {dt * 1e3:.2f} ms  "
              f"({2 / 3 * n ** 3 / dt / 1e12:.2f} TFLOP/s)  err={err:.2e}", flush=True)


if __name__ == "__main__":
    main()
