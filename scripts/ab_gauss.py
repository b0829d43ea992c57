"""A/B timing of GaussSolver variants in ONE process (interleaved rounds)."""
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2048
dev = torch.device("cuda:0")
src = gelim.random_system(n, seed=1234, device=dev)
variants = {}
# schedule is read from the environment when a plan is created
# plans read GELIM_* at creation; GELIM_PANEL_IO is read at every enqueue, so
# the io variants run eagerly with the variable set around each solve
VARIANTS = {
    "fused+narrow io=2": {"GELIM_SCHEDULE": "fused", "GELIM_LOOKAHEAD": "0", "GELIM_PANEL_IO": "2", "GELIM_NARROW": "1"},
    "fused+narrow io=1": {"GELIM_SCHEDULE": "fused", "GELIM_LOOKAHEAD": "0", "GELIM_PANEL_IO": "1", "GELIM_NARROW": "1"},
    "fused+narrow io=0": {"GELIM_SCHEDULE": "fused", "GELIM_LOOKAHEAD": "0", "GELIM_PANEL_IO": "0", "GELIM_NARROW": "1"},
    "fused prologue": {"GELIM_SCHEDULE": "fused", "GELIM_LOOKAHEAD": "0", "GELIM_PANEL_IO": "1", "GELIM_NARROW": "0"},
    "classic": {"GELIM_SCHEDULE": "classic", "GELIM_LOOKAHEAD": "0", "GELIM_PANEL_IO": "0", "GELIM_NARROW": "0"},
}
for name, env in VARIANTS.items():
    os.environ.update(env)
    variants[name] = gelim.GaussSolver(n, "hip", device=dev, use_graph=False)
if "--pivot" in sys.argv:
    variants["hip-pivot"] = gelim.GaussSolver(n, "hip-pivot", device=dev)
res = {k: [] for k in variants}
for s in variants.values():
    for _ in range(3):
        s.solve(src)
os.environ["GELIM_PANEL_IO"] = "0"
torch.cuda.synchronize()
for rnd in range(5):
    for k, s in variants.items():
        os.environ.update(VARIANTS.get(k, {}))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            x = s.solve(src)
        torch.cuda.synchronize()
        res[k].append((time.perf_counter() - t0) / 5)
        assert gelim.ops.gauss.error_metric(x) < 1e-6, k
for k, v in res.items():
    print(f"{k:28s} median {statistics.median(v)*1e3:8.3f} ms  min {min(v)*1e3:8.3f} ms")
