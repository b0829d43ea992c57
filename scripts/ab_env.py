"""A/B timing of per-launch environment knobs (GELIM_PANEL_IO, GELIM_NARROW,
...) on the fused blocked-LU solve, interleaved in ONE process, eager launches.

  python scripts/ab_env.py N 'NAME:VAR=V,VAR=V' 'NAME:VAR=V' ...
"""
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

n = int(sys.argv[1])
variants = {}
for spec in sys.argv[2:]:
    name, _, kv = spec.partition(":")
    variants[name] = dict(x.split("=", 1) for x in kv.split(",") if x)
dev = torch.device("cuda:0")
src = gelim.random_system(n, seed=1234, device=dev)
solver = gelim.GaussSolver(n, "hip", device=dev, use_graph=False)
res = {k: [] for k in variants}
errs = {}
base = dict(os.environ)
for rnd in range(7):
    for k, env in variants.items():
        os.environ.clear()
        os.environ.update(base)
        os.environ.update(env)
        for _ in range(2 if rnd == 0 else 0):
            solver.solve(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            x = solver.solve(src)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 5)
        errs[k] = gelim.ops.gauss.error_metric(x)
for k, v in res.items():
    print(f"n={n} {k:20s} median {statistics.median(v)*1e3:8.3f} ms  min {min(v)*1e3:8.3f} ms  err {errs[k]:.2e}",
          flush=True)
