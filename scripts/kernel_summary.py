"""Per-kernel totals of a rocprofv3 kernel trace (csv), divided by the
number of solves in the run: python scripts/kernel_summary.py trace.csv [solves]"""
import collections
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    solves = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tot = collections.defaultdict(lambda: [0, 0])
    grid = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("gelim::", "").split("(")[0]
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[name][0] += 1
        tot[name][1] += d
        g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        grid[(name, g)][0] += 1
        grid[(name, g)][1] += d
    all_ns = sum(v[1] for v in tot.values())
    print(f"{'kernel':58s} {'calls/solve':>11s} {'ms/solve':>9s} {'avg_us':>8s}")
    for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"{k[:58]:58s} {c / solves:11.1f} {d / solves / 1e6:9.3f} {d / c / 1e3:8.1f}")
    print(f"{'sum of kernel time':58s} {'':11s} {all_ns / solves / 1e6:9.3f}")
    print("top (kernel, workgroups):")
    for k, (c, d) in sorted(grid.items(), key=lambda kv: -kv[1][1])[:12]:
        print(f"  {k[0][:40]:40s} wg={k[1]:7d} calls={c:5d} avg={d / c / 1e3:8.1f} us")


if __name__ == "__main__":
    main()
