"""Host issue time vs GPU time of the distributed schedules on ONE rank.

For each schedule: (a) the solve as it runs (host issues while the GPU
executes), (b) the host time to issue the factorisation loop
(`last_issue_s`), and (c) the GPU-only time of the same factorisation: a
bounded spin kernel (gelim_gpu_probe_kernel, 150 ms) holds the main stream
while the whole schedule is queued behind it, so the events around the
schedule time the GPU with no host gap.  (c) < (a)'s factor part means the
host issue is on the critical path.

  python scripts/dist_issue.py [--n 8192] [--pg]    (--pg: one-rank RCCL group)
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--pg", action="store_true")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None, help="also write the JSON here")
    a = ap.parse_args()
    import torch

    import gelim
    from gelim import _native
    from gelim.parallel import DistributedGauss, DistributedRBT
    from gelim.parallel import comm as C
    from gelim.utils.tensors import ptr

    if a.pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        comm = C.init_from_env(backend="nccl", force_pg=True)
    else:
        comm = C.init_from_env()
    dev = comm.device
    lib = _native.lib()
    words = torch.zeros(2, dtype=torch.int32, device=dev)
    out = {"n": a.n, "backend": comm.backend}

    def gpu_only(factor):
        """Factorisation queued behind a 150 ms spin: GPU-only time."""
        torch.cuda.synchronize(dev)
        words.zero_()
        _native.check(lib.gelim_gpu_probe_kernel(torch.cuda.current_stream(dev).cuda_stream, ptr(words), 0,
                                                 15_000_000), "spin")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        factor()
        issue = time.perf_counter() - t0
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) * 1e-3, issue

    def as_runs(factor):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        factor()
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    # DistributedRBT: the distributed schedule on one rank, eager and graph-replayed
    for tag, graph in (("rbt_eager", False), ("rbt", True)):
        d = DistributedRBT(comm, a.n, single_fast_path=False, graph=graph)
        loc = d.generate_random(seed=99)
        d.solve_(loc)
        d.solve_(loc)  # (graph: the second solve captures)
        rows = []
        for _ in range(a.reps):
            wall = as_runs(lambda: d.factor_(loc))
            issue_wall = d.last_issue_s
            g, issue_q = gpu_only(lambda: d.factor_(loc))
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            d.solve_(loc)
            torch.cuda.synchronize(dev)
            rows.append({"factor_wall_s": wall, "factor_issue_s": issue_wall, "factor_gpu_only_s": g,
                         "solve_s": time.perf_counter() - t0, "steps": d.last_steps})
        out[tag] = {"blocks": d.nb, "graph": d.graph, "runs": rows,
                    "issue_us_per_block": min(r["factor_issue_s"] for r in rows) / d.nb * 1e6,
                    "gpu_us_per_block": min(r["factor_gpu_only_s"] for r in rows) / d.nb * 1e6}
        d.close()
        del d, loc

    # DistributedGauss: lookahead schedule, every block a broadcast panel (tail = 0) and the default
    for tag, tail in (("gauss_tail0", 0), ("gauss", None)):
        dg = DistributedGauss(comm, a.n, tail=tail)
        G = dg._panel_blocks(use_tail=True)
        rows = []
        for _ in range(a.reps):
            loc = dg.generate_random(seed=99)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            dg.solve_(loc)
            torch.cuda.synchronize(dev)
            rows.append({"solve_s": time.perf_counter() - t0, "factor_issue_s": dg.last_issue_s})
            loc = dg.generate_random(seed=99)

            def panels():  # _factor_wide's set-up, then the panels alone (no tail solve: it syncs)
                dg._info.zero_()
                dg._ws.zero_()
                dg._factor_lookahead(loc, G, None)

            g, iq = gpu_only(panels)
            rows[-1].update(panels_gpu_only_s=g, issue_queued_s=iq)
        out[tag] = {"panels": G, "runs": rows,
                    "issue_us_per_panel": min(r["factor_issue_s"] for r in rows) / max(1, G) * 1e6,
                    "gpu_us_per_panel": min(r["panels_gpu_only_s"] for r in rows) / max(1, G) * 1e6}
        del dg
    print(json.dumps(out, indent=1), flush=True)
    if a.out:
        Path(a.out).write_text(json.dumps(out, indent=1))
    C.destroy()


if __name__ == "__main__":
    main()
