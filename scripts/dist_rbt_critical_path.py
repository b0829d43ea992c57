"""Critical-path estimate of the distributed randomised solver
(parallel/dist_rbt.py) at P ranks, from a one-rank kernel trace of its
distributed schedule (scripts/dist_rbt_prof.py under rocprofv3
--kernel-trace; one rank owns every block, so its main stream runs the whole
chain and its side stream all trailing updates).

Per block k the owner of k+1 (main stream) needs panel k -- the column
broadcast X_k and the inverse broadcast D_k -- and then updates block k+1 and
ships it.  D_k leaves after the inverse, X_k before it, so

  chain_k = max(bcast(X_k), inv_k + bcast(D_k)) + [W + column update of k+1 + pack]

with the kernel times measured here and an RCCL broadcast model
bcast(bytes) = latency + bytes / bandwidth.  Every rank's side stream applies
panel k to ITS columns, ~1/P of the one-rank side work per block; a block
costs max(chain_k, side_k / P).  Solves: per direction np / (128 P)
super-blocks of one all_reduce (latency) + a super-block solve + a GEMV.

  python scripts/dist_rbt_critical_path.py gpurun_out/drbt/run_results.db 8192
"""
import sqlite3
import sys


def load(path: str):
    con = sqlite3.connect(path)
    return con.execute("select name, start, end, stream_id, grid_x from kernels order by start").fetchall()


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    ks = load(path)
    inv = [k for k in ks if "diag_inv_kernel" in k[0]]
    nb = n // 128
    if len(inv) < nb:
        raise SystemExit(f"only {len(inv)} inverse dispatches in the trace")
    last = inv[-nb:]  # the last distributed-schedule solve
    t0, t1 = last[0][1], last[-1][2]
    # the solve's window: from its first inverse back to its transform, forward to the last kernel
    win = [k for k in ks if k[1] >= t0 - 2_000_000 and k[2] <= t1 + 50_000_000]
    main_stream = last[0][3]
    inv_us = [(k[2] - k[1]) / 1e3 for k in last]
    # per-block main-stream work between consecutive inverses (W, block update, packs)
    chain_other = []
    side_work = []
    for i in range(nb - 1):
        a, b = last[i][2], last[i + 1][1]
        seg = [k for k in win if k[1] >= a and k[2] <= b + 1]
        chain_other.append(sum((k[2] - k[1]) / 1e3 for k in seg if k[3] == main_stream))
        side_work.append(sum((k[2] - k[1]) / 1e3 for k in seg if k[3] != main_stream))
    chain_other.append(0.0)
    side_work.append(0.0)
    span_1rank = (win[-1][2] - win[0][1]) / 1e3
    solve_k = [k for k in win if k[1] > t1]
    ss = [(k[2] - k[1]) / 1e3 for k in solve_k if "super_solve" in k[0]]
    gv = [(k[2] - k[1]) / 1e3 for k in solve_k if "gemv_acc" in k[0]]
    mean = lambda v: sum(v) / len(v) if v else 0.0  # noqa: E731
    print(f"# one-rank trace: {len(win)} kernels in the last schedule solve, span {span_1rank / 1e3:.2f} ms")
    print(f"# inverse: mean {mean(inv_us):.1f} us, min {min(inv_us):.1f}, max {max(inv_us):.1f} (x{nb})")
    print(f"# main-stream work between inverses (W, block update, packs): mean {mean(chain_other):.1f} us")
    print(f"# side-stream work per block at one rank: mean {mean(side_work):.1f} us, total "
          f"{sum(side_work) / 1e3:.2f} ms")
    print(f"# super-block solve {mean(ss):.1f} us, gemv {mean(gv):.1f} us (one rank: S = 128)")
    print()
    print("P  bcast-lat(us) bcast-BW(GB/s)  chain(ms)  side-bound(ms)  factor(ms)  solves(ms)  total(ms)")
    for P in (2, 4, 8):
        for lat, bw in ((15.0, 100.0), (25.0, 50.0)):
            chain = side = fac = 0.0
            for k in range(nb):
                xbytes = (n - 128 * k) * 128 * 8
                bx = lat + xbytes / (bw * 1e3)  # us
                bd = lat + 128 * 128 * 8 / (bw * 1e3)
                c = max(bx, inv_us[k] + bd) + chain_other[k]
                s = side_work[k] / P
                chain += c
                side += s
                fac += max(c, s)
            ns = n // (128 * P)
            # forward + backward per apply, one apply + one correction typical
            solves = 2 * 2 * ns * (lat + mean(ss) * P + mean(gv))
            print(f"{P}  {lat:12.0f} {bw:14.0f} {chain / 1e3:10.2f} {side / 1e3:14.2f} {fac / 1e3:11.2f} "
                  f"{solves / 1e3:11.2f} {(fac + solves) / 1e3:10.2f}")


if __name__ == "__main__":
    main()
