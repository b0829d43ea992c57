"""Distributed Gauss (parallel/dist_gauss.py) on ONE GPU with P emulated
ranks: wall time of the second solve of a random n x n system and its error.
P = 1 is the real single-rank code path (no communication); P > 1 checks
the multi-rank schedule at full size (ranks share the card: not a scaling
number).

  python scripts/time_dist.py P n [block] [--no-lookahead]
"""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.parallel import DistributedGauss, run_emulated  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
P, n = int(args[0]), int(args[1])
block = int(args[2]) if len(args) > 2 else None
la = "--no-lookahead" not in sys.argv


def body(c):
    dg = DistributedGauss(c, n, block=block, lookahead=la)
    out = []
    for _ in range(2):
        loc = dg.generate_random(seed=99)
        torch.cuda.synchronize()
        c.barrier()
        t0 = time.perf_counter()
        x = dg.solve_(loc)
        torch.cuda.synchronize()
        c.barrier()
        out.append(time.perf_counter() - t0)
    return out[-1], gelim.ops.gauss.error_metric(x)


res = run_emulated(P, body, device="cuda:0", timeout_s=600)
t = max(r[0] for r in res)
print(f"dist_gauss P={P} n={n} block={block or 256} lookahead={la}: {t * 1e3:.2f} ms "
      f"({2 / 3 * n ** 3 / t * 1e-12:.2f} TFLOP/s), err {res[0][1]:.2e}", flush=True)
