"""Per-kernel duration summary from a rocprofv3 SQLite output (rocpd schema,
the default output format of rocprofv3 in ROCm 7): name, calls, mean / min
duration (us).  Usage: python scripts/rocpd_kernels.py <run_results.db> [filter]"""
import sqlite3
import sys


def summary(path: str, filt: str = ""):
    con = sqlite3.connect(path)
    rows = con.execute("select name, count(*), avg(end - start), min(end - start), sum(end - start) "
                       "from kernels group by name order by sum(end - start) desc").fetchall()
    out = []
    for name, calls, avg, mn, tot in rows:
        if filt and filt not in name:
            continue
        out.append((name, calls, avg / 1e3, mn / 1e3, tot / 1e3))
    return out


if __name__ == "__main__":
    for name, calls, avg, mn, tot in summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""):
        print(f"{calls:6d} {avg:10.2f} {mn:10.2f} {tot:12.1f}  {name[:110]}")
