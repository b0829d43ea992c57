"""Critical-path view of a rocprofv3 kernel trace of
`scripts/one_rank_of_p.py --factor-only`: the last factorisation (from the
last drbt_transform_kernel on), per-kernel totals, per-queue busy time, and
the main queue's timeline for a few blocks (kernel, start, duration, gap
before it) -- where each chain step's time goes.

  python scripts/orp_trace_summary.py run_kernel_trace.csv [first_block] [blocks]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
qk = "Queue_Id" if "Queue_Id" in rows[0] else "Stream_Id"
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             r["Kernel_Name"].replace("gelim::(anonymous namespace)::", "").replace("void ", "").split("(")[0][-48:],
             r[qk]) for r in rows)
first = [i for i, k in enumerate(ks) if "drbt_transform" in k[2]][-1]
ks = ks[first:]
t0, t1 = ks[0][0], max(k[1] for k in ks)
print(f"factorisation span {(t1 - t0) / 1e6:.3f} ms, {len(ks)} kernels")
per = defaultdict(lambda: [0, 0.0])
for s, e, n, q in ks:
    per[n][0] += 1
    per[n][1] += (e - s) / 1e3
for n, (c, us) in sorted(per.items(), key=lambda kv: -kv[1][1])[:12]:
    print(f"  {us / 1e3:8.3f} ms {c:5d} x {us / c:8.1f} us  {n}")
byq = defaultdict(float)
for s, e, n, q in ks:
    byq[q] += (e - s) / 1e6
print("busy per queue (ms):", {q: round(v, 3) for q, v in byq.items()})
invq = [q for s, e, n, q in ks if "diag_inv" in n][0]
main = [k for k in ks if k[3] == invq]
invs = [i for i, k in enumerate(main) if "diag_inv" in k[2]]
b0 = int(sys.argv[2]) if len(sys.argv) > 2 else len(invs) // 2
nbk = int(sys.argv[3]) if len(sys.argv) > 3 else 3
lo, hi = invs[b0], invs[min(b0 + nbk, len(invs) - 1)]
print(f"main queue {invq}, blocks {b0}..{b0 + nbk} (gap = idle time before the kernel on this queue):")
prev = main[lo - 1][1] if lo > 0 else main[lo][0]
for s, e, n, q in main[lo - 4:hi + 1]:
    print(f"  t={(s - t0) / 1e3:9.1f} us  dur={(e - s) / 1e3:7.1f}  gap={(s - prev) / 1e3:6.1f}  {n}")
    prev = e
steps = [(main[invs[i + 1]][0] - main[invs[i]][0]) / 1e3 for i in range(len(invs) - 1)]
steps.sort()
print(f"inverse-to-inverse on the main queue: median {steps[len(steps) // 2]:.1f} us, "
      f"p10 {steps[len(steps) // 10]:.1f}, p90 {steps[9 * len(steps) // 10]:.1f}")
inv = sorted((e - s) / 1e3 for s, e, n, q in main if "diag_inv" in n)
print(f"inverse durations: median {inv[len(inv) // 2]:.1f} us, min {inv[0]:.1f}, max {inv[-1]:.1f}")
