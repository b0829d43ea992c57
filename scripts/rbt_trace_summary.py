"""Summarise a rocprofv3 kernel trace of the last hip-rbt factorisation:
span, per-kernel time, per-queue busy time, and how much of the diagonal
inverses ran under a side-stream GEMM.

  python scripts/rbt_trace_summary.py run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", r.get("Stream_Id", "?")))
      for r in rows]
ks.sort()
# the last factorisation: from the last rbt_matrix_kernel on
starts = [i for i, k in enumerate(ks) if "rbt_matrix_kernel" in k[2]]
ks = ks[starts[-1]:]
t0, t1 = ks[0][0], max(k[1] for k in ks)
print(f"factorisation span {(t1 - t0) / 1e6:.3f} ms, {len(ks)} kernels")
per = defaultdict(lambda: [0, 0.0])
for s, e, n, q in ks:
    key = n.replace("gelim::(anonymous namespace)::", "").replace("void ", "").split("(")[0][-60:]
    per[key][0] += 1
    per[key][1] += (e - s) / 1e3
for key, (c, us) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print(f"  {us / 1e3:8.3f} ms {c:5d} x {us / c:8.1f} us  {key}")
byq = defaultdict(float)
for s, e, n, q in ks:
    byq[q] += (e - s) / 1e6
print("busy per queue (ms):", {q: round(v, 3) for q, v in byq.items()})
diag = [(s, e) for s, e, n, q in ks if "diag_inv" in n]
big = [(s, e) for s, e, n, q in ks if "dgemm" in n]
under = 0.0
for s, e in diag:
    for gs, ge in big:
        lo, hi = max(s, gs), min(e, ge)
        if hi > lo:
            under += (hi - lo)
tot = sum(e - s for s, e in diag)
print(f"diagonal inverses: {tot / 1e6:.3f} ms total, {under / 1e6:.3f} ms overlapped with some dgemm")
