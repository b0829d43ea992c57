"""Critical-path model of the distributed randomised solver
(parallel/dist_rbt.py) at P ranks, from measured one-GPU kernel times
(scripts/dist_rbt_prof.py --micro, profiles/dgemm_thin_r4.txt) and an RCCL
model bcast(bytes) = latency + bytes / bandwidth.

Factorisation, per 128-column block k (m = rows below block k):
  the owner of block k+1 (main stream), once panel k has arrived:
    W = Dinv_k A[k, k+1]  +  column update of block k+1  +  pack of column k+1
  then the column broadcast X_{k+1} leaves, the inverse of block k+1 runs
  under it, and its 128 x 128 broadcast D_{k+1} follows:
    chain_k = t_W + t_upd(m) + t_pack(m) + max(bcast(X), t_inv + bcast(D))
  every rank's side stream applies panel k to its own columns (~1/P of the
  trailing update); a block costs max(chain_k, side_k).
Solves (per apply): ns = np / (128 P) super-blocks per direction, each one
all_reduce (latency + S doubles) + the persistent block solve of P blocks +
one local GEMV; refinement = 1 + corrections applies, each followed by a
residual (local |A||x| mat-vec + an all_reduce of 2 np doubles).
Setup: the butterfly transform (local) and the all_gather of the super-blocks
(np x 128 P doubles) and of the inverses (np x 128).
Host issue (round 5, profiles/dist_issue_r5.md): the host must issue a
block's ~15 launches and 2 collectives; a block then costs
max(chain_k, side_k, issue) -- issue = 255 us eagerly through
torch.distributed, 176 us eagerly through libgelim's RCCL communicators, 28 us
replaying the captured hipGraph (the default; the graph launch overlaps the
GPU).

  python scripts/dist_rbt_critical_path.py [n]
"""
import sys

# measured on one MI355X (us); profiles/dist_rbt_8rank_critical_path.md
T_INV = 57.0                       # 128 x 128 Gauss-Jordan inverse (one workgroup, two steps per barrier)
T_SS = {1: 8.3, 2: 12.1, 4: 19.2, 8: 34.4}   # persistent block solve of P blocks
T_GEMV = 4.6                       # 8192 x 128 local GEMV
T_PACK_8192 = 8.1                  # column pack, 8192 x 128 (8.4 MB)
T_TRANSFORM_8192 = 120.0           # one-rank butterfly transform, 8192^2 (scales 1/P)


def t_gemm_thin(m: int) -> float:
    """m x 128 x 128 fp64 GEMM (dgemm.hip LDS kernel): 9.5 us at m = 1024, 11.5
    at 8064 (profiles/dgemm_thin_r4.txt)."""
    return 9.5 + 2.0 * max(0, m - 1024) / 7040


ISSUE_US = {"torch-eager": 255.0, "native-eager": 176.0, "graph": 28.0}


def model(n: int, P: int, lat: float, bw: float, corrections: int = 2, issue: float = 0.0) -> dict:
    NB = 128
    np_ = -(-n // (512 * P)) * 512 * P
    nb = np_ // NB
    us_per_byte = 1.0 / (bw * 1e3)    # GB/s -> bytes per us
    chain = side = fac = 0.0
    for k in range(nb - 1):
        m = np_ - NB * (k + 1)
        xb = m * NB * 8
        c = t_gemm_thin(NB) + t_gemm_thin(m) + T_PACK_8192 * m / 8192 + 2.0 + max(
            lat + xb * us_per_byte, T_INV + lat + NB * NB * 8 * us_per_byte)
        # side: panel k on this rank's ~(np - 128 k) / P trailing columns: a W
        # GEMM and an m x cols x 128 GEMM at ~40 TF/s
        cols = (np_ - NB * (k + 1)) / P
        s = 2 * t_gemm_thin(NB) + 2.0 * m * cols * NB / 40e6
        chain += c
        side += s
        fac += max(c, s, issue)
    fac += T_INV
    S = NB * P
    ns = np_ // S
    t_ss = T_SS.get(P, T_SS[8] * P / 8)
    # the applies are graph-replayed too: ~4 launches + 1 all_reduce per super-block
    per_apply = 2 * ns * max(lat + S * 8 * us_per_byte + t_ss + T_GEMV, issue / 4)
    resid = lat + 2 * np_ * 8 * us_per_byte + 10.0
    solves = (1 + corrections) * (per_apply + resid)
    gather = (np_ * S * 8 + np_ * NB * 8) * us_per_byte * (P - 1) / P + 2 * lat
    setup = T_TRANSFORM_8192 * (np_ / 8192) ** 2 / P + gather
    return {"np": np_, "chain": chain, "side": side, "factor": fac, "solves": solves, "setup": setup,
            "total": fac + solves + setup}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    print(f"# n = {n}; inverse {T_INV} us, block solves {T_SS} us, GEMV {T_GEMV} us, pack {T_PACK_8192} us/8.4 MB")
    for name, iss in ISSUE_US.items():
        print(f"# host issue: {name} ({iss:.0f} us per block)")
        print("P  lat(us) BW(GB/s)  chain  side-bound  factor  solves  setup   total (ms)")
        for P in (2, 4, 8):
            for lat, bw in ((15.0, 100.0), (25.0, 50.0)):
                r = model(n, P, lat, bw, issue=iss)
                print(f"{P}  {lat:6.0f} {bw:8.0f} {r['chain'] / 1e3:7.2f} {r['side'] / 1e3:10.2f} "
                      f"{r['factor'] / 1e3:7.2f} {r['solves'] / 1e3:7.2f} {r['setup'] / 1e3:6.2f} {r['total'] / 1e3:7.2f}")


if __name__ == "__main__":
    main()
