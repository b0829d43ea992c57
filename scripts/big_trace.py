"""Timeline of the LAST wide-panel solve in a rocprofv3 kernel trace
(biglu.hip / plan.hip enqueue_big): span, per-kernel totals split by
stream, the leaf chain (sum of leaf durations vs the span) and how much of
the side stream's GEMM time overlapped the leaves.

  python scripts/big_trace.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gelim::", "")
    depth, out = 0, []
    for ch in name:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:44]


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                 f'{r.get("Queue_Id", "?")}/{r.get("Stream_Id", "?")}') for r in rows)
    # the last solve: from the first leaf after the second-to-last tail_gemv
    tg = [i for i, e in enumerate(ev) if "tail_gemv" in e[2]]
    prev = tg[-2] if len(tg) > 1 else -1
    first = min(i for i, e in enumerate(ev) if i > prev and "leaf_kernel" in e[2])
    last = max(i for i, e in enumerate(ev) if "backsub_persist" in e[2])
    w = ev[first:last + 1]
    t0, t1 = w[0][0], max(e[1] for e in w)
    print(f"last solve: {len(w)} dispatches, span {(t1 - t0) / 1e6:.3f} ms")
    agg = defaultdict(lambda: [0, 0])
    for s, e, n, q in w:
        agg[(n, q)][0] += 1
        agg[(n, q)][1] += e - s
    print(f"  {'kernel':44s} {'queue/stream':>12s} {'calls':>6s} {'total ms':>9s} {'avg us':>8s}")
    for (n, q), (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {n:44s} {q:>12s} {c:6d} {d / 1e6:9.3f} {d / c / 1e3:8.1f}")
    leaves = [(s, e) for s, e, n, _ in w if "leaf_kernel" in n]
    lt = sum(e - s for s, e in leaves)
    print(f"leaf chain: {len(leaves)} leaves, {lt / 1e6:.3f} ms of leaf time "
          f"({100 * lt / (t1 - t0):.0f}% of the span), avg {lt / len(leaves) / 1e3:.1f} us")
    # GEMM time that ran while some leaf was running
    gem = [(s, e) for s, e, n, _ in w if "dgemm" in n]
    ov = 0
    for s, e in gem:
        for ls, le in leaves:
            ov += max(0, min(e, le) - max(s, ls))
    gt = sum(e - s for s, e in gem)
    print(f"dgemm: {gt / 1e6:.3f} ms total, {ov / 1e6:.3f} ms of it under a leaf")
    lend = max(e for s, e in leaves)
    print(f"after the last leaf: {(t1 - lend) / 1e6:.3f} ms (tail system + back substitution)")


if __name__ == "__main__":
    main()
