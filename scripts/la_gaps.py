"""Critical-stream idle gaps of the last wide-panel solve in a rocprofv3
kernel trace of the lookahead schedule (plan.hip enqueue_big): total idle
time of the leaf stream between consecutive kernels, by kernel pair, and
the side stream's per-panel first-part latency.

  python scripts/la_gaps.py gpurun_out/pbig_la64/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gelim::", "")
    return name.split("(")[0].split("<")[0][-28:]


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r.get("Queue_Id"))
                for r in rows)
    tg = [i for i, e in enumerate(ev) if "tail_gemv" in e[2]]
    prev = tg[-2] if len(tg) > 1 else -1
    first = min(i for i, e in enumerate(ev) if i > prev and "leaf_kernel" in e[2])
    w = ev[first:]
    q0 = w[0][3]
    crit = [e for e in w if e[3] == q0]
    side = [e for e in w if e[3] != q0]
    gaps = defaultdict(lambda: [0, 0])
    for a, b in zip(crit, crit[1:]):
        gaps[(a[2], b[2])][0] += b[0] - a[1]
        gaps[(a[2], b[2])][1] += 1
    print(f"crit busy {sum(e[1] - e[0] for e in crit) / 1e6:.3f} ms, idle {sum(g for g, _ in gaps.values()) / 1e6:.3f} ms")
    for (a, b), (g, c) in sorted(gaps.items(), key=lambda x: -x[1][0])[:6]:
        print(f"  {g / 1e6:8.3f} ms over {c:4d} gaps  {a} -> {b}")
    agg = defaultdict(lambda: [0, 0])
    for s, e, n, _ in side:
        agg[n][0] += 1
        agg[n][1] += e - s
    print("side kernels:", ", ".join(f"{n} {c}x {d / c / 1e3:.1f} us" for n, (c, d) in agg.items()))


if __name__ == "__main__":
    main()
