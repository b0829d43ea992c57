"""Wall time per GaussSolver.solve (hip backend, fp64, partial pivoting) for
the orders in argv, random U[-1,1) systems with b = A(1..n): the solve is
replayed from its captured graph, timed between two synchronisations.

  python scripts/time_solver.py 2048 4096 8192 [--reps 5]
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
    ap.add_argument("--pivot", default="partial")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for n in args.n:
        aug = gelim.random_system(n, seed=n, device=dev)
        s = gelim.GaussSolver(n, backend="hip", pivot=args.pivot, device=dev)
        t0 = time.perf_counter()
        x = s.solve(aug, check=True)
        torch.cuda.synchronize()
        first = time.perf_counter() - t0
        s.solve(aug)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            x = s.solve(aug)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        err = gelim.ops.gauss.error_metric(x)
        print(f"n={n}: {dt * 1e3:.3f} ms/solve ({2 / 3 * n ** 3 / dt / 1e12:.2f} TFLOP/s), first call "
              f"(capture+instantiate+run) {first * 1e3:.1f} ms, err={err:.2e}, info={s.info()}", flush=True)
        del s, aug, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
