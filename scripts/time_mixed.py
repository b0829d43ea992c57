"""Wall time of the mixed-precision solve (RBT + fp32 no-pivot MFMA LU + fp64
refinement) vs the fp64 partial-pivoting engine, random systems.

  python scripts/time_mixed.py 2048 4096 8192 [--reps 3]
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402

args = [int(a) for a in sys.argv[1:] if a.isdigit()]
dev = torch.device("cuda:0")
for n in args:
    aug = gelim.random_system(n, seed=n, device=dev)
    for backend in ("hip-mixed", "hip"):
        s = gelim.GaussSolver(n, backend=backend, device=dev)
        x = s.solve(aug, check=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            x = s.solve(aug, check=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        extra = f", {s.last_steps} corrections, fallback={s.last_fallback}" if backend == "hip-mixed" else ""
        print(f"n={n} {backend}: {dt * 1e3:.2f} ms, err {gelim.ops.gauss.error_metric(x):.2e}{extra}", flush=True)
        s.close()
