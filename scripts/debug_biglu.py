"""Step-by-step check of the wide-panel LU composition on one GPU: runs the
driver sequence of plan.hip (enqueue_big) through the exposed primitives
(leaf, laswp+TRSM, dgemm) and compares every step with a plain fp64 torch
implementation of the same blocked algorithm.  Prints the first step whose
result diverges.

  python scripts/debug_biglu.py [n] [K]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim import _native  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

LW, NB = 32, 256


def ref_leaf(A, c0, kend):
    """LAPACK-style leaf on rows [c0, n) x cols [c0, c0+32) + interchanges of
    all other columns + TRSM of the leaf's U rows (cols right of the leaf)."""
    n = A.shape[0]
    P = A[c0:, c0:c0 + LW].clone()
    lu_, piv = torch.linalg.lu_factor(P)
    perm = list(range(n - c0))
    for j, pj in enumerate(piv.tolist()):
        perm[j], perm[pj - 1] = perm[pj - 1], perm[j]
    perm = torch.tensor(perm)
    sub = A[c0:].clone()
    A[c0:] = sub[perm]
    A[c0:, c0:c0 + LW] = lu_
    L = torch.tril(lu_[:LW], -1) + torch.eye(LW, dtype=A.dtype)
    A[c0:c0 + LW, c0 + LW:kend] = torch.linalg.solve_triangular(L, A[c0:c0 + LW, c0 + LW:kend], upper=False,
                                                                unitriangular=True)


def main() -> None:
    pos = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(pos[0]) if pos else 300
    K = int(pos[1]) if len(pos) > 1 else 64
    dev = torch.device("cuda:0")
    lda = (n + 2 + 7) // 8 * 8
    aug = gelim.random_system(n, seed=3, device=dev).cpu()
    H = torch.zeros(n, lda, dtype=torch.float64)
    H[:, :n + 1] = aug[:, :n + 1]
    G = H.to(dev)
    lib = _native.lib()
    sh = stream_handle(dev)
    ipiv = torch.zeros(n + 64, dtype=torch.int32, device=dev)
    pairs = torch.zeros(200, dtype=torch.int32, device=dev)
    info = torch.zeros(4, dtype=torch.int32, device=dev)

    def cmp(what):
        torch.cuda.synchronize()
        d = (G.cpu()[:, :n + 1] - H[:, :n + 1]).abs().max().item()
        print(f"{what}: max|gpu-ref| = {d:.3e}", flush=True)
        if d > 1e-6 * max(1.0, H[:, :n + 1].abs().max().item()):
            bad = ((G.cpu()[:, :n + 1] - H[:, :n + 1]).abs() > 1e-8).nonzero()
            print("  first bad entries (row, col):", bad[:8].tolist())
            sys.exit(1)

    def dgemm(c, a, b, M, N, Kk):
        # c, a, b: (row, col) offsets into G
        rc = lib.gelim_gpu_dgemm(ptr(G) + 8 * (c[0] * lda + c[1]), lda, ptr(G) + 8 * (a[0] * lda + a[1]), lda,
                                 ptr(G) + 8 * (b[0] * lda + b[1]), lda, M, N, Kk, -1.0, sh)
        _native.check(rc, "dgemm")

    shared_ws = "--shared-ws" in sys.argv
    ws = torch.zeros(int(lib.gelim_gpu_leaf_workspace_bytes()) // 8, dtype=torch.float64, device=dev)
    leaf = 0
    for k in range(0, K, NB):
        kend = min(k + NB, K)
        for c0 in range(k, kend, LW):
            if shared_ws:
                rc = lib.gelim_gpu_leaf_factor_ws(ptr(G) + 8 * (c0 * lda + c0), lda, n - c0, c0, 1, ptr(ipiv),
                                                  ptr(pairs), ptr(info), ptr(ws), leaf, sh)
            else:
                rc = lib.gelim_gpu_leaf_factor(ptr(G) + 8 * (c0 * lda + c0), lda, n - c0, c0, 1, ptr(ipiv),
                                               ptr(pairs), ptr(info), sh)
            leaf += 1
            _native.check(rc, "leaf")
            rc = lib.gelim_gpu_laswp_trsm(ptr(G) + 8 * (c0 * lda), lda, c0, c0, c0 + LW, n + 1, kend, n - c0,
                                          ptr(pairs), sh)
            _native.check(rc, "laswp")
            ref_leaf(H, c0, kend)
            cmp(f"leaf c0={c0}")
            c1 = c0 + LW
            if c1 < kend:
                dgemm((c1, c1), (c1, c0), (c0, c1), n - c1, kend - c1, LW)
                H[c1:, c1:kend] -= H[c1:, c0:c1] @ H[c0:c1, c1:kend]
                cmp(f"  gemm_a c0={c0}")

        for r in range(k, kend, LW):
            rc = lib.gelim_gpu_laswp_trsm(ptr(G) + 8 * (r * lda), lda, r, 0, kend, n + 1, n + 1, n - r, None, sh)
            _native.check(rc, "trsm")
            if r + LW < kend:
                dgemm((r + LW, kend), (r + LW, r), (r, kend), kend - r - LW, n + 1 - kend, LW)
        L11 = torch.tril(H[k:kend, k:kend], -1) + torch.eye(kend - k, dtype=H.dtype)
        H[k:kend, kend:n + 1] = torch.linalg.solve_triangular(L11, H[k:kend, kend:n + 1], upper=False,
                                                              unitriangular=True)
        cmp(f"U12 k={k}")
        dgemm((kend, kend), (kend, k), (k, kend), n - kend, n + 1 - kend, kend - k)
        H[kend:, kend:n + 1] -= H[kend:, k:kend] @ H[k:kend, kend:n + 1]
        cmp(f"outer k={k}")
    print("composition ok")
    # the plan's own working matrix after a solve of the same system
    import ctypes as C
    import os
    os.environ["GELIM_BIG_TAIL"] = str(n - K)
    solver = gelim.GaussSolver(n, backend="hip", device=dev, use_graph=False)
    xs = solver.solve(aug.to(dev))
    torch.cuda.synchronize()
    W = torch.zeros(n, lda, dtype=torch.float64)
    wp = lib.gelim_gauss_plan_work(C.c_void_p(solver._plan))
    _native.check(lib.gelim_gpu_memcpy_d2h(W.data_ptr(), wp, n * lda * 8, None), "d2h")
    torch.cuda.synchronize()
    Gh = G.cpu()
    d = (W[:, :n + 1] - Gh[:, :n + 1]).abs()
    print(f"plan work vs composition: max diff {d.max().item():.3e}; bad rows {d.max(1).values.gt(1e-6).nonzero()[:10].flatten().tolist()}"
          f" bad cols {d.max(0).values.gt(1e-6).nonzero()[:10].flatten().tolist()}")
    xr = torch.linalg.solve(aug[:, :n], aug[:, n])
    print(f"plan x vs torch: {(xs.cpu() - xr).abs().max().item():.3e}")
    # the tail system through a nested solver on the strided view, as the plan does
    Gv = G[K:, K:]
    xt = gelim.GaussSolver(n - K, backend="hip", device=dev).solve(Gv, check=True)
    rt = torch.linalg.solve(H[K:, K:n], H[K:, n])
    print(f"tail via strided view: max|x-ref| = {(xt.cpu() - rt).abs().max().item():.3e}")
    Gc = G[K:, K:n + 1].contiguous()
    xc = gelim.GaussSolver(n - K, backend="hip", device=dev).solve(Gc, check=True)
    print(f"tail via contiguous copy: max|x-ref| = {(xc.cpu() - rt).abs().max().item():.3e}")
    print(f"plan x[K:] vs python tail: {(xs.cpu()[K:] - xt.cpu()).abs().max().item():.3e}")
    y = H[:K, n] - H[:K, K:n] @ xt.cpu()
    x1 = torch.linalg.solve_triangular(torch.triu(H[:K, :K]), y[:, None], upper=True)[:, 0]
    print(f"plan x[:K] vs torch block backsub: {(xs.cpu()[:K] - x1).abs().max().item():.3e}; "
          f"torch block x vs torch full: {(torch.cat([x1, xt.cpu()]) - xr).abs().max().item():.3e}")
    print("plan x[K:K+8]", xs.cpu()[K:K + 8].tolist())
    print("tail x[:8]   ", xt.cpu()[:8].tolist())


if __name__ == "__main__":
    main()
