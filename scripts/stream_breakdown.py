"""Per-stream breakdown of the LAST solve in a rocprofv3 kernel trace
(rocpd SQLite): the window runs back from the end of the trace to the first
device-wide idle gap longer than `gap_us` (default 300: the host's
synchronisation between solves).  Per stream: busy time, kernel count, and the kernels by total
time; the idle gaps of the busiest stream (its critical path is its busy time
plus its waits).

  python scripts/stream_breakdown.py run_results.db [gap_us]
"""
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    gap_ns = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 300e3
    con = sqlite3.connect(path)
    ks = con.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    t0 = ks[0][1]
    horizon = ks[-1][2]  # earliest start seen so far, walking backwards
    for k in reversed(ks):
        if horizon - k[2] > gap_ns:
            t0 = horizon
            break
        horizon = min(horizon, k[1])
    win = [k for k in ks if k[1] >= t0]
    t1 = max(k[2] for k in win)
    print(f"# window {(t1 - t0) / 1e3:.1f} us, {len(win)} kernels")
    by_stream = defaultdict(list)
    for k in win:
        by_stream[k[3]].append(k)
    for sid, lst in sorted(by_stream.items(), key=lambda kv: -sum(k[2] - k[1] for k in kv[1])):
        busy = sum(k[2] - k[1] for k in lst)
        print(f"stream {sid}: {len(lst)} kernels, busy {busy / 1e3:.1f} us ({100 * busy / (t1 - t0):.0f} % of the window)")
        agg = defaultdict(lambda: [0, 0])
        for k in lst:
            a = agg[k[0][:100]]
            a[0] += 1
            a[1] += k[2] - k[1]
        for name, (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:10]:
            print(f"   {c:5d} x {tot / c / 1e3:8.2f} us = {tot / 1e3:9.1f} us  {name}")
        gaps = [(lst[i + 1][1] - lst[i][2]) for i in range(len(lst) - 1) if lst[i + 1][1] > lst[i][2]]
        if gaps:
            print(f"   idle gaps: {len(gaps)}, total {sum(gaps) / 1e3:.1f} us, mean {sum(gaps) / len(gaps) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
