"""Critical-path model of DistributedGauss (partial pivoting, parallel/
dist_gauss.py) at P ranks for n = 8192 ... 32768, from one-MI355X
measurements: the single-GPU solve time (bench gauss_{n}_1gpu_s), the leaf
chain's per-column cost, the K = 256 trailing-GEMM rate and an RCCL model
bcast(bytes) = latency + bytes / bandwidth.

Schedule (1-D column block-cyclic, D = 256, lookahead on two streams): the
last T = 2048 columns are the tail system (one all_gather + the single-GPU
2048 engine on every rank); the first n - T columns are G = (n - T) / 256
broadcast panels.  Block step g (owner o = g mod P) -- the chain:
    bcast(panel g: m x 256 + row lists)  ->  owner of g+1: apply panel g to
    block g+1 (laswp + TRSM + (m-256) x 256 x 256 GEMM)  ->  factor block g+1
    (8 leaves of m x 32 + in-panel K = 32 updates)  ->  bcast(panel g+1)
Off the chain: each rank's side-stream trailing update (1/P of the total
GEMM flops), which competes with the chain for CUs (capped grid).

Per step:  chain_g = bcast(m_g) + apply(m_g) + factor(m_g)
           side_g  = (2 m_g (n_g / P) 256) / R_gemm
  step_g = max(chain_g, side_g);  total = sum_g step_g + tail + back substitution.
The pivot chain (leaves) does not shrink with P: every column needs one
global arg-max.  The bandwidth term is itemised: bytes broadcast per rank.

  python scripts/dist_gauss_critical_path.py [n ...]
"""
import sys

D = 256        # panel width
T = 2048       # tail system
LEAF_US_PER_COL = {2048: 2.73, 4096: 3.07, 8192: 2.93, 16384: 3.91, 32768: 3.12}  # leaf_shape_r4.txt (2-wave)
R_GEMM_TF = 45.0      # K = 256 trailing update on the capped side grid (gemm_microbench.txt: 44-54 TF/s)
R_APPLY_TF = 30.0     # the owner's (m - 256) x 256 x 256 apply (thin; gemm_microbench.txt)
T_TAIL_MS = 3.9       # 2048 engine (bench dist_gauss_2048_tail_engine_s)
ONE_GPU_S = {8192: 0.0295, 16384: 0.112, 32768: 0.664}  # bench gauss_{n}_1gpu_s / README (round 5)


def leaf_us(m: int) -> float:
    keys = sorted(LEAF_US_PER_COL)
    k = min(keys, key=lambda x: abs(x - m))
    return LEAF_US_PER_COL[k]


def model(n: int, P: int, lat_us: float, bw_gbs: float) -> dict:
    G = (n - T) // D
    chain = side = total = 0.0
    leaves = bcast = 0.0
    bytes_per_rank = 0.0
    for g in range(G):
        m = n - g * D
        nb_cols = n - (g + 1) * D
        t_b = lat_us + m * D * 8 / (bw_gbs * 1e3)
        t_apply = 5.0 + 2.0 * (m - D) * D * D / (R_APPLY_TF * 1e6)
        t_fac = 8 * 32 * leaf_us(m) + 8 * 6.0  # 8 leaves + their laswp/TRSM/K=32 updates
        c = t_b + t_apply + t_fac
        s = 2.0 * m * (nb_cols / P) * D / (R_GEMM_TF * 1e6)
        chain += c
        side += s
        total += max(c, s)
        leaves += t_fac
        bcast += t_b
        bytes_per_rank += m * D * 8
    # tail: all_gather of the trailing 2048 system + the 2048 engine; back
    # substitution over ceil((n - T) / (D P)) super-blocks
    tail = lat_us + T * T * 8 / (bw_gbs * 1e3) + T_TAIL_MS * 1e3
    nsuper = -(-(n - T) // (D * P))
    backsub = nsuper * (2 * lat_us + 150.0)
    total += tail + backsub
    one = ONE_GPU_S.get(n)
    return {"n": n, "P": P, "lat_us": lat_us, "bw_GBs": bw_gbs, "panels": G,
            "leaf_chain_ms": leaves / 1e3, "bcast_on_chain_ms": bcast / 1e3,
            "bcast_GB_per_rank": bytes_per_rank / 1e9, "side_ms": side / 1e3, "tail_ms": tail / 1e3,
            "backsub_ms": backsub / 1e3, "total_ms": total / 1e3,
            "one_gpu_ms": one * 1e3 if one else None,
            "speedup": (one * 1e3) / (total / 1e3) if one else None}


def main() -> None:
    ns = [int(a) for a in sys.argv[1:]] or [8192, 16384, 32768]
    print(f"{'n':>6} {'P':>2} {'lat':>4} {'BW':>4} {'panels':>6} {'leaves':>8} {'bcast':>7} {'GB/rank':>7} "
          f"{'side':>7} {'tail':>5} {'total':>8} {'1 GPU':>7} {'speedup':>7}   (ms unless noted)")
    for n in ns:
        for P in (2, 4, 8):
            for lat, bw in ((15, 100), (25, 50)):
                r = model(n, P, lat, bw)
                print(f"{n:6d} {P:2d} {lat:4d} {bw:4d} {r['panels']:6d} {r['leaf_chain_ms']:8.1f} "
                      f"{r['bcast_on_chain_ms']:7.1f} {r['bcast_GB_per_rank']:7.2f} {r['side_ms']:7.1f} "
                      f"{r['tail_ms']:5.1f} {r['total_ms']:8.1f} {r['one_gpu_ms'] or 0:7.1f} "
                      f"{r['speedup'] or 0:7.2f}x")


if __name__ == "__main__":
    main()
