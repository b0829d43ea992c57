"""Wall time per hip-pivot solve (the reference's per-pivot algorithm on the
GPU: one pivot launch + one elimination launch per column, graph-replayed),
fp64 and fp32, for the orders in argv.

  python scripts/time_pivot.py 1024 2048 [--reps 5]
"""
import argparse
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="+")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for n in args.n:
        aug = gelim.random_system(n, seed=n, device=dev)
        for dtype in (torch.float64, torch.float32):
            s = gelim.GaussSolver(n, backend="hip-pivot", dtype=dtype, device=dev)
            a = aug.to(dtype)
            x = s.solve(a)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.reps):
                x = s.solve(a)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.reps
            print(f"n={n} {str(dtype)[6:]}: {dt * 1e3:.3f} ms/solve, err={gelim.ops.gauss.error_metric(x):.3e}",
                  flush=True)
            s.close()


if __name__ == "__main__":
    main()
