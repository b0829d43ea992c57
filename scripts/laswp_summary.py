"""Median device time of the laswp kernel per grid size in a rocprofv3 kernel trace."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    if "laswp" in r["Kernel_Name"]:
        d[int(r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(d.items()):
    v = sorted(v)
    print(f"grid {k}: {len(v)} calls, median {v[len(v) // 2] / 1e3:.1f} us")
