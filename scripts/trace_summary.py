"""Summarise a rocprofv3 kernel trace: per-kernel stats and the timeline of
the last N dispatches (busy vs idle, concurrency)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
tr = list(csv.DictReader(open(path)))


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").replace("gelim::", "")
    depth, out = 0, []
    for ch in name:  # drop the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:48]


ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in tr)
ev = ev[-last:]
t0 = ev[0][0]
span = ev[-1][1] - t0
# union of busy intervals
busy = 0
cur_s, cur_e = ev[0][0], ev[0][1]
for s, e, _ in ev[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"last {len(ev)} dispatches: span {span/1e3:.1f} us, device busy (union) {busy/1e3:.1f} us, idle {100*(1-busy/span):.1f}%")
agg = defaultdict(lambda: [0, 0])
for s, e, n in ev:
    agg[n][0] += 1
    agg[n][1] += e - s
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {n:48s} {c:5d} calls {d/1e3:9.1f} us total {d/c/1e3:7.2f} us avg")
nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 40
print(f"first {nshow} dispatches of the window (start offset us, duration us):")
for s, e, n in ev[:nshow]:
    print(f"  {(s-t0)/1e3:9.2f} {(e-s)/1e3:7.2f}  {n}")
