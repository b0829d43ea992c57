"""Overlap in the LAST DistributedGauss solve of a rocprofv3 kernel trace of
scripts/time_dist.py: per-kernel totals by stream, the leaf chain, and how
much of the trailing-update kernels (dgemm, panel TRSM, row movement) ran
while a leaf was running -- the two-stream lookahead of
parallel/dist_gauss.py.

  python scripts/dist_trace.py gpurun_out/pdist/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from big_trace import short  # noqa: E402


def overlap(a, b):
    """Total time of intervals a that lies under the union of intervals b."""
    b = sorted(b)
    merged = []
    for s, e in b:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    tot = 0
    for s, e in a:
        for ms, me in merged:
            if me <= s:
                continue
            if ms >= e:
                break
            tot += min(e, me) - max(s, ms)
    return tot


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 f'{r.get("Queue_Id", "?")}/{r.get("Stream_Id", "?")}') for r in rows)
    inits = [i for i, e in enumerate(ev) if "init_random" in e[2]]
    start = inits[-1] + 1 if inits else 0
    w = [e for e in ev[start:]]
    leaves = [(s, e) for s, e, n, _ in w if "leaf_kernel" in n]
    first = min(s for s, _ in leaves)
    w = [x for x in w if x[0] >= first]
    t0, t1 = w[0][0], max(x[1] for x in w)
    print(f"last solve: {len(w)} dispatches from its first leaf, span {(t1 - t0) / 1e6:.3f} ms")
    agg = defaultdict(lambda: [0, 0])
    for s, e, n, q in w:
        agg[(n, q)][0] += 1
        agg[(n, q)][1] += e - s
    print(f"  {'kernel':44s} {'queue/stream':>12s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s}")
    for (n, q), (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:16]:
        print(f"  {n:44s} {q:>12s} {c:6d} {d / 1e6:9.3f} {d / c / 1e3:8.1f}")
    lt = sum(e - s for s, e in leaves)
    print(f"leaf chain: {len(leaves)} leaves, {lt / 1e6:.3f} ms ({100 * lt / (t1 - t0):.0f}% of the span)")
    for tag in ("dgemm", "panel_trsm", "laswp_panel"):
        ks = [(s, e) for s, e, n, _ in w if tag in n]
        if ks:
            tot = sum(e - s for s, e in ks)
            print(f"{tag:12s}: {tot / 1e6:.3f} ms total, {overlap(ks, leaves) / 1e6:.3f} ms of it under a leaf")


if __name__ == "__main__":
    main()
