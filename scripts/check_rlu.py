"""GPU check + A/B timing of the resident LU (GELIM_SCHEDULE=resident forces it
up to n = 2048; the auto default uses it up to 1024) against the fused step
schedule and torch.linalg.solve.

  python scripts/check_rlu.py [--time] [n ...]
"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

dev = torch.device("cuda:0")
args = [a for a in sys.argv[1:] if not a.startswith("--")]
sizes = [int(a) for a in args] or [1, 2, 7, 16, 17, 33, 64, 100, 511, 512, 513, 1000, 1024, 1025, 1500, 2047, 2048]


def solver(n, sched, pivot="partial", graph=False):
    os.environ["GELIM_SCHEDULE"] = sched
    try:
        return gelim.GaussSolver(n, backend="hip", pivot=pivot, device=dev, use_graph=graph)
    finally:
        os.environ.pop("GELIM_SCHEDULE", None)


worst = 0.0
for n in sizes:
    aug = gelim.random_system(n, seed=n, device=dev)
    s = solver(n, "resident")
    x = s.solve(aug)
    info = s.info()
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    rel = ((x - ref).abs().max() / ref.abs().max()).item()
    err = gelim.ops.gauss.error_metric(x)
    worst = max(worst, rel)
    print(f"n={n:5d} info={info} rel_vs_torch={rel:.3e} err_metric={err:.3e}", flush=True)
    assert info == 0 and rel < 1e-8, (n, info, rel)

# synthetic internal system with the zero-pivot rule: exact (-0.5, 0, ..., 0.5)
for n in (8, 16, 100, 2048):
    s = solver(n, "resident", pivot="zero")
    x, bn = s.solve(gelim.synthetic_system(n, device=dev), return_bnorm=True)
    xc = x.cpu()
    assert abs(xc[0] + 0.5) < 1e-12 and abs(xc[-1] - 0.5) < 1e-12 and xc[1:-1].abs().max() < 1e-12, n
    print(f"synthetic n={n} ok", flush=True)

# singular
n = 64
aug = gelim.random_system(n, seed=3, device=dev)
aug[:, 20] = 0.0
s = solver(n, "resident")
s.solve(aug)
print("singular info:", s.info())
assert s.info() > 0

print(f"all ok, worst rel {worst:.3e}", flush=True)

if "--time" in sys.argv:
    for n in (512, 1024, 2048):
        aug = gelim.random_system(n, seed=1234, device=dev)
        res = {}
        for sched in ("resident", "fused"):
            s = solver(n, sched)
            for _ in range(3):
                s.solve(aug)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                s.solve(aug)
            torch.cuda.synchronize()
            res[sched] = (time.perf_counter() - t0) / 10 * 1e3
        print(f"n={n}: " + "  ".join(f"{k} {v:.3f} ms" for k, v in res.items()), flush=True)
