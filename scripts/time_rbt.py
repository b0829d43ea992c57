"""Wall time of hip-rbt solves (median of 5 after 2 warm-ups) for the orders
in argv; for kernel traces: rocprofv3 --kernel-trace -- python3 scripts/time_rbt.py 8192"""
import statistics
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(a) for a in sys.argv[1:]] or [8192]:
    aug = gelim.random_system(n, seed=n + 31, device=dev)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
    for _ in range(2):
        s.solve(aug)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x = s.solve(aug)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    print(f"n={n} hip-rbt {statistics.median(ts) * 1e3:.3f} ms (min {min(ts) * 1e3:.3f}), corrections {s.last_steps}, "
          f"error {gelim.ops.gauss.error_metric(x):.2e}", flush=True)
    s.close()
