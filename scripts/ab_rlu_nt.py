"""A/B of the resident LU's workgroup shape on the n = 2048 solve (round 4):
the default hybrid (fused steps + 1024-row resident tail), the resident LU
over the whole system with 512 threads (4 register slots) and with 1024
threads (2 slots, GELIM_RLU_NT=1024).  Interleaved in one process.

  python scripts/ab_rlu_nt.py [n]
"""
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
dev = torch.device("cuda:0")
src = gelim.random_system(n, seed=1234, device=dev)
ref = torch.linalg.solve(src[:, :n], src[:, n])
variants = {"hybrid": ({}, {}), "resident512": ({"GELIM_SCHEDULE": "resident"}, {}),
            "resident1024": ({"GELIM_SCHEDULE": "resident"}, {"GELIM_RLU_NT": "1024"})}
solvers = {}
for k, (cenv, _) in variants.items():
    os.environ.update(cenv)
    solvers[k] = gelim.GaussSolver(n, "hip", device=dev, use_graph=False)
    for v in cenv:
        del os.environ[v]
res = {k: [] for k in variants}
errs = {}
for rnd in range(7):
    for k, (_, renv) in variants.items():
        os.environ.update(renv)
        s = solvers[k]
        for _ in range(2 if rnd == 0 else 0):
            s.solve(src)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            x = s.solve(src)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 5)
        errs[k] = ((x - ref).abs().max() / ref.abs().max()).item()
        for v in renv:
            del os.environ[v]
for k, v in res.items():
    print(f"n={n} {k:14s} median {statistics.median(v)*1e3:8.3f} ms  min {min(v)*1e3:8.3f} ms  "
          f"rel diff vs torch {errs[k]:.2e}", flush=True)
