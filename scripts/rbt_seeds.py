"""How robust is the randomised engine's refinement?  One process, one GPU:
64 random systems each at n = 2048 and 8192, solved by the single-GPU
`hip-rbt` engine and by the one-rank distributed schedule (DistributedRBT,
single_fast_path=False).  Reports the correction-count histogram, the final
componentwise backward error (in units of eps64) and the fallback rate.

  python scripts/rbt_seeds.py [--seeds 64] [--sizes 2048 8192] [--out FILE]

The acceptance rule (GaussSolver / gelim_mixed_solve, dist_rbt.solve_):
componentwise backward error <= 4 eps; a stall or too many corrections hand the
system to partial pivoting.  Reference metric: the error computation of
Pthreads/Version-1/gauss_external_input.c:308-315."""
from __future__ import annotations

import argparse
import collections
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402
from gelim.parallel import DistributedRBT  # noqa: E402
from gelim.parallel.comm import Communicator  # noqa: E402

EPS = torch.finfo(torch.float64).eps


def summarise(tag: str, recs: list[dict]) -> str:
    hist = collections.Counter(r["steps"] for r in recs)
    fb = sum(1 for r in recs if r["fallback"])
    berr = sorted(r["berr"] / EPS for r in recs if r["berr"] is not None)
    over4 = sum(1 for b in berr if b > 4.0)
    ge4 = sum(1 for r in recs if r["steps"] >= 4)
    worst = max(recs, key=lambda r: (r["steps"], r["berr"] or 0.0))
    return (f"{tag:28s} systems {len(recs):3d}  corrections {dict(sorted(hist.items()))}  "
            f">=4 corrections {ge4} ({100.0 * ge4 / len(recs):.1f} %)  final berr > 4 eps {over4}  fallbacks {fb}  "
            f"berr/eps median {berr[len(berr) // 2]:.2f} max {berr[-1]:.2f}  "
            f"worst seed {worst['seed']} ({worst['steps']} corrections, {worst['berr'] / EPS:.1f} eps)  "
            f"mean time {sum(r['t'] for r in recs) / len(recs) * 1e3:.2f} ms")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=64)
    ap.add_argument("--sizes", type=int, nargs="+", default=[2048, 8192])
    ap.add_argument("--out", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    comm = Communicator(0, 1, dev, "none")
    lines, raw = [], {}
    for n in a.sizes:
        single = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
        dist = DistributedRBT(comm, n, single_fast_path=False)
        rs, rd = [], []
        for seed in range(a.seeds):
            aug = gelim.random_system(n, seed=seed, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x = single.solve(aug)
            torch.cuda.synchronize()
            rs.append({"seed": seed, "steps": single.last_steps, "berr": single.last_berr,
                       "fallback": single.last_fallback, "t": time.perf_counter() - t0,
                       "error": gelim.ops.gauss.error_metric(x)})
            loc = dist.scatter_from_global(aug)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x = dist.solve_(loc)
            torch.cuda.synchronize()
            rd.append({"seed": seed, "steps": dist.last_steps, "berr": dist.last_berr,
                       "fallback": dist.last_fallback, "t": time.perf_counter() - t0,
                       "error": gelim.ops.gauss.error_metric(x)})
            del aug, loc
        single.close()
        dist.close()
        for tag, recs in ((f"hip-rbt n={n}", rs), (f"DistributedRBT 1 rank n={n}", rd)):
            line = summarise(tag, recs)
            print(line, flush=True)
            lines.append(line)
            raw[tag] = recs
    if a.out:
        Path(a.out).write_text("\n".join(lines) + "\n")
    if a.json:
        Path(a.json).write_text(json.dumps(raw))


if __name__ == "__main__":
    main()
