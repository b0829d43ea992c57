"""Wide-panel LU (n > 2048; biglu.hip + dgemm.hip) and the fp64 MFMA GEMM,
against plain fp64 PyTorch references of the same ops."""
import pytest
import torch

from conftest import GOLDEN_ERROR

pytestmark = pytest.mark.gpu


def _dgemm(gelim, C, A, B, alpha, cap=None):
    from gelim import _native
    from gelim.utils.tensors import ptr, row_major_ld, stream_handle

    M, N = C.shape
    K = A.shape[1]
    args = (ptr(C), row_major_ld(C), ptr(A), row_major_ld(A), ptr(B), row_major_ld(B), M, N, K, alpha)
    if cap is None:
        rc = _native.lib().gelim_gpu_dgemm(*args, stream_handle(C.device))
    else:
        rc = _native.lib().gelim_gpu_dgemm_capped(*args, cap, stream_handle(C.device))
    _native.check(rc, "dgemm")


@pytest.mark.parametrize("M,N,K", [(128, 128, 16), (256, 384, 256), (300, 517, 32), (129, 1, 2),
                                   (1000, 2049, 64), (64, 64, 30)])
@pytest.mark.parametrize("alpha", [-1.0, 1.0])
@pytest.mark.parametrize("cap", [None, 8, 224])
def test_dgemm_matches_torch(gelim, cuda, M, N, K, alpha, cap):
    """Plain launch, and the persistent capped form (512-thread workgroups,
    two tiles each, odd tile counts leaving an idle half) on 8 / 224 CUs."""
    torch.manual_seed(M * 7 + N + K)
    ldn = N + 1 + (N + 1) % 2  # even, > N (the dgemm contract)
    Cf = torch.randn(M, ldn, dtype=torch.float64, device=cuda)
    Af = torch.randn(M, K + 2, dtype=torch.float64, device=cuda)
    Bf = torch.randn(K, ldn, dtype=torch.float64, device=cuda)
    C, A, B = Cf[:, :N], Af[:, :K], Bf[:, :N]
    ref = C + alpha * (A @ B)
    C0 = Cf.clone()
    _dgemm(gelim, C, A, B, alpha, cap)
    torch.cuda.synchronize()
    assert torch.allclose(C, ref, rtol=1e-12, atol=1e-11 * K)
    assert torch.equal(Cf[:, N:], C0[:, N:])  # padding untouched


@pytest.mark.parametrize("group", [4, 8])
@pytest.mark.parametrize("M,N,K", [(1300, 1000, 32), (2100, 3000, 64), (200, 700, 16)])
@pytest.mark.parametrize("cap", [0, 224])
def test_dgemm_grouped_tile_order(gelim, cuda, M, N, K, group, cap):
    """The grouped tile order (gelim_gpu_dgemm_grouped: runs of g tile rows, the
    last run short: 11 / 17 / 2 tile rows of 128, or of 64 for the thin-tile
    path) still covers every tile exactly once, plain and persistent."""
    from gelim import _native
    from gelim.utils.tensors import stream_handle

    torch.manual_seed(M + N + K)
    ldn = N + 2
    Cf = torch.randn(M, ldn, dtype=torch.float64, device=cuda)
    A = torch.randn(M, K, dtype=torch.float64, device=cuda)
    Bf = torch.randn(K, ldn, dtype=torch.float64, device=cuda)
    C, B = Cf[:, :N], Bf[:, :N]
    ref = C - A @ B
    rc = _native.lib().gelim_gpu_dgemm_grouped(C.data_ptr(), C.stride(0), A.data_ptr(), A.stride(0), B.data_ptr(),
                                               B.stride(0), M, N, K, -1.0, cap, group, stream_handle(C.device))
    _native.check(rc, "dgemm")
    torch.cuda.synchronize()
    assert torch.allclose(C, ref, rtol=1e-12, atol=1e-11 * K)


def test_dgemm_rejects_odd_k(gelim, cuda):
    C = torch.zeros(16, 16, dtype=torch.float64, device=cuda)
    A = torch.zeros(16, 3, dtype=torch.float64, device=cuda)
    B = torch.zeros(3, 16, dtype=torch.float64, device=cuda)
    with pytest.raises(gelim.GelimError):
        _dgemm(gelim, C, A, B, -1.0)


@pytest.mark.parametrize("m", [32, 100, 1024, 1025, 3000, 8192])
def test_leaf_factor_matches_lapack(gelim, cuda, m):
    """One 32-column leaf over P = ceil(m/1024) workgroups: pivots equal
    LAPACK's getrf, factors match to rounding, pairs reproduce the row
    order."""
    from gelim import _native
    from gelim.utils.tensors import ptr, stream_handle

    torch.manual_seed(m)
    ld = 40
    P = torch.randn(m, ld, dtype=torch.float64)
    Pg = P.to(cuda)
    ipiv = torch.zeros(32, dtype=torch.int32, device=cuda)
    pairs = torch.zeros(1 + 4 * 32, dtype=torch.int32, device=cuda)
    info = torch.zeros(4, dtype=torch.int32, device=cuda)
    rc = _native.lib().gelim_gpu_leaf_factor(ptr(Pg), ld, m, 0, 1, ptr(ipiv), ptr(pairs), ptr(info),
                                             stream_handle(cuda))
    _native.check(rc, "leaf_factor")
    torch.cuda.synchronize()
    assert info.cpu()[1].item() == 0
    lu_, piv_ref = torch.linalg.lu_factor(P[:, :32])
    assert torch.equal(ipiv.cpu().long() + 1, piv_ref.long())
    assert torch.allclose(Pg.cpu()[:, :32], lu_, rtol=1e-10, atol=1e-10)
    assert torch.equal(Pg.cpu()[:, 32:], P[:, 32:])
    # the pair list is the net permutation of the LAPACK interchanges
    perm = list(range(m))
    for j, pj in enumerate(piv_ref.tolist()):
        perm[j], perm[pj - 1] = perm[pj - 1], perm[j]
    pr = pairs.cpu().tolist()
    moved = {pr[1 + 2 * e]: pr[2 + 2 * e] for e in range(pr[0])}
    for dst in range(m):
        assert moved.get(dst, dst) == perm[dst]


def test_laswp_trsm_matches_torch(gelim, cuda):
    from gelim import _native
    from gelim.utils.tensors import ptr, stream_handle

    torch.manual_seed(1)
    n, c0 = 300, 64
    ncols = n + 1
    A = torch.randn(n, ncols + 1, dtype=torch.float64)
    m = n - c0
    perm = torch.randperm(m)[:40]
    tgt = torch.arange(m)
    src_rows = tgt.clone()
    src_rows[perm] = perm[torch.randperm(40)]  # a permutation of 40 rows
    pl = [(int(d), int(s)) for d, s in zip(tgt.tolist(), src_rows.tolist()) if d != s]
    pairs = torch.zeros(1 + 4 * 32, dtype=torch.int32)
    pairs[0] = len(pl)
    for e, (d, s) in enumerate(pl):
        pairs[1 + 2 * e], pairs[2 + 2 * e] = d, s
    Ag = A.to(cuda)
    rc = _native.lib().gelim_gpu_laswp_trsm(ptr(Ag[c0:]), A.shape[1], c0, c0, c0 + 32, ncols, ncols, n - c0,
                                            ptr(pairs.to(cuda)), stream_handle(cuda))
    _native.check(rc, "laswp_trsm")
    torch.cuda.synchronize()
    L2 = torch.tril(A[c0:c0 + 32, c0:c0 + 32], -1) + torch.eye(32, dtype=torch.float64)
    ref2 = A.clone()
    ref2[c0:, :c0] = A[c0:][src_rows][:, :c0]
    ref2[c0:, c0 + 32:] = A[c0:][src_rows][:, c0 + 32:]
    ref2[c0:c0 + 32, c0 + 32:ncols] = torch.linalg.solve_triangular(L2, ref2[c0:c0 + 32, c0 + 32:ncols],
                                                                    upper=False, unitriangular=True)
    assert torch.allclose(Ag.cpu()[:, :ncols], ref2[:, :ncols], rtol=1e-11, atol=1e-11)


def _check_solve(gelim, cuda, n, seed, rtol=1e-8):
    aug = gelim.random_system(n, seed=seed, device=cuda)
    x = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    torch.cuda.synchronize()
    assert torch.allclose(x, ref, rtol=rtol, atol=rtol * n), (x - ref).abs().max().item()
    assert gelim.ops.gauss.error_metric(x) < 1e-6


@pytest.mark.parametrize("n", [2049, 2500, 3000, 4096, 8192])
def test_big_solver_vs_torch(gelim, cuda, n):
    _check_solve(gelim, cuda, n, seed=n + 11)


@pytest.mark.parametrize("n", [300, 700, 1000])
def test_big_solver_small_tail(gelim, cuda, monkeypatch, n):
    """GELIM_BIG_TAIL=256 runs the wide-panel engine on small systems: several
    outer panels, leaves with 1 workgroup, a short tail."""
    monkeypatch.setenv("GELIM_BIG_TAIL", "256")
    _check_solve(gelim, cuda, n, seed=n + 3)


def test_big_solver_multi_workgroup_leaf_ties(gelim, cuda, monkeypatch):
    """Integer-valued system with many equal |a| candidates across
    workgroups: the global arg-max must resolve ties to the lowest row
    (LAPACK / the reference's strict '>') or the solution drifts."""
    n = 3100
    g = torch.Generator().manual_seed(5)
    A = torch.randint(-3, 4, (n, n), generator=g).double()
    A += torch.eye(n, dtype=torch.float64) * 0.5
    x0 = torch.arange(1, n + 1, dtype=torch.float64)
    aug = torch.cat([A, (A @ x0)[:, None]], 1).to(cuda)
    x = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    P, L, U = torch.linalg.lu(A)
    ref = torch.linalg.solve(A, A @ x0)
    assert torch.allclose(x.cpu(), ref, rtol=1e-7, atol=1e-6)


def test_big_zero_rule_verify_pattern(gelim, cuda):
    """The internal programs' zero-pivot rule through the wide-panel engine:
    synthetic 2*min(i+1,j+1) system, exact pattern."""
    n = 2300
    aug = gelim.synthetic_system(n, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", pivot="zero", device=cuda)
    x, bn = s.solve(aug, return_bnorm=True)
    expect = torch.zeros(n, dtype=torch.float64)
    expect[0], expect[-1] = -0.5, 0.5
    eb = torch.full((n,), 0.5, dtype=torch.float64)
    eb[0] = 0.0
    assert torch.allclose(x.cpu(), expect, rtol=0, atol=1e-11)
    assert torch.allclose(bn.cpu(), eb, rtol=0, atol=1e-11)


@pytest.mark.parametrize("zero_col", [40, 700, 2900])
def test_big_singular_column(gelim, cuda, zero_col):
    """A zero column inside a leaf (40, 700) or inside the tail system (2900):
    info is the 1-based column of the first zero pivot."""
    n = 3000
    aug = gelim.random_system(n, seed=5, device=cuda)
    aug[:, zero_col] = 0.0
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    s.solve(aug)
    assert s.info() == zero_col + 1


def test_big_graph_replay_two_plans(gelim, cuda):
    n = 2600
    s1 = gelim.GaussSolver(n, backend="hip", device=cuda)
    s2 = gelim.GaussSolver(n, backend="hip", device=cuda)
    a1 = gelim.random_system(n, seed=1, device=cuda)
    a2 = gelim.random_system(n, seed=2, device=cuda)
    x1 = s1.solve(a1).clone()
    x2 = s2.solve(a2).clone()
    for _ in range(3):  # interleaved replays of both graphs
        assert torch.equal(s1.solve(a1), x1)
        assert torch.equal(s2.solve(a2), x2)
    torch.cuda.synchronize()
    for x, a in ((x1, a1), (x2, a2)):
        assert torch.allclose(x, torch.linalg.solve(a[:, :n], a[:, n]), rtol=1e-8, atol=1e-8 * n)


@pytest.mark.parametrize("name", [k for k in GOLDEN_ERROR if k in ("orsreg_1", "sherman5", "saylr4", "sherman3")])
def test_big_golden_errors(gelim, cuda, name):
    """The four reference matrices with n > 2048 now run the wide-panel
    engine: same accuracy class as the reference's fp64 OpenMP program."""
    A = gelim.utils.io.load_fixture(name)
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    x = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    err = gelim.ops.gauss.error_metric(x)
    assert err <= max(20 * GOLDEN_ERROR[name], 1e-14), (name, err)


def test_memplus_blocked(gelim, cuda):
    """memplus (n = 17758, the one reference matrix the reference never
    benchmarked): solved by the blocked engine on one GPU.  No golden value
    exists, so the oracle is rocSOLVER's fp64 solve of the same system
    (parity unpinned against the reference)."""
    A = gelim.utils.io.load_fixture("memplus")
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    del A
    x = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    err = gelim.ops.gauss.error_metric(x)
    xr = torch.linalg.solve(aug[:, :n], aug[:, n])
    err_ref = gelim.ops.gauss.error_metric(xr)
    assert err <= max(20 * err_ref, 1e-12), (err, err_ref)


@pytest.mark.parametrize("la", ["0", "1"])
@pytest.mark.parametrize("n", [700, 1500, 2600, 3100])
def test_big_schedules_agree(gelim, cuda, monkeypatch, la, n):
    """Serial (graph-captured) and lookahead (side stream on a capped grid:
    the CU count less 64, and never fewer free CUs than the first leaf needs)
    schedules of the wide-panel engine, several outer panels each
    (GELIM_BIG_TAIL=256): same pivots, so the same solution to rounding."""
    monkeypatch.setenv("GELIM_BIG_TAIL", "256")
    monkeypatch.setenv("GELIM_BIG_LOOKAHEAD", la)
    _check_solve(gelim, cuda, n, seed=n + 29)


def test_big_lookahead_replays_identically(gelim, cuda, monkeypatch):
    """The eager lookahead schedule is deterministic: replays are bitwise equal."""
    monkeypatch.setenv("GELIM_BIG_TAIL", "512")
    n = 3000
    aug = gelim.random_system(n, seed=3, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x = s.solve(aug).clone()
    for _ in range(3):
        assert torch.equal(s.solve(aug), x)


def test_laswp_panel_matches_sequential(gelim, cuda):
    """laswp_panel = the leaves' pair lists applied in order (each list a
    gather-then-scatter permutation), only on the requested column ranges."""
    from gelim import _native
    from gelim.utils.tensors import ptr, stream_handle

    torch.manual_seed(4)
    n, c0, nl, slot = 500, 96, 3, 1 + 4 * 32 + 3
    ncols = n + 1
    A = torch.randn(n, ncols + 1, dtype=torch.float64)
    pairs = torch.zeros(nl * slot, dtype=torch.int32)
    ref = A.clone()
    lb, le, rb, re = 10, 80, 300, ncols
    cols = list(range(lb, le)) + list(range(rb, re))
    for l in range(nl):
        base = c0 + 32 * l
        m = n - base
        sel = torch.randperm(m)[:50]
        src = torch.arange(m)
        src[sel] = sel[torch.randperm(50)]
        pl = [(d, s) for d, s in enumerate(src.tolist()) if d != s][:64]
        pairs[l * slot] = len(pl)
        for e, (d, s) in enumerate(pl):
            pairs[l * slot + 1 + 2 * e], pairs[l * slot + 2 + 2 * e] = d, s
        old = ref.clone()
        for d, s in pl:
            ref[base + d, cols] = old[base + s, cols]
    net = torch.zeros(1 + 2 * 64 * nl, dtype=torch.int32, device=cuda)
    for cap in (0, 2):  # one workgroup per 64 columns / a 2-workgroup grid-stride loop
        Ag = A.to(cuda)
        rc = _native.lib().gelim_gpu_laswp_panel(ptr(Ag), A.shape[1], n, c0, nl, ptr(pairs.to(cuda)), slot, lb, le,
                                                 rb, re, cap, stream_handle(cuda))
        _native.check(rc, "laswp_panel")
        torch.cuda.synchronize()
        assert torch.equal(Ag.cpu(), ref)
        # the composed permutation (compose + gather/scatter) moves the same rows
        Ag = A.to(cuda)
        rc = _native.lib().gelim_gpu_laswp_net(ptr(Ag), A.shape[1], n, c0, nl, ptr(pairs.to(cuda)), slot, lb, le, rb,
                                               re, ptr(net), cap, stream_handle(cuda))
        _native.check(rc, "laswp_net")
        torch.cuda.synchronize()
        assert torch.equal(Ag.cpu(), ref)
        assert 0 < int(net[0]) <= 64 * nl


@pytest.mark.parametrize("nb,ncols", [(256, 1000), (32, 70), (160, 33), (256, 8193)])
@pytest.mark.parametrize("cap", [0, 3])
def test_panel_trsm_matches_torch(gelim, cuda, nb, ncols, cap):
    """The one-launch U12 = L11^-1 A12 of an outer panel (nb rows, unit lower
    L11) against torch's triangular solve."""
    from gelim import _native
    from gelim.utils.tensors import ptr, stream_handle

    torch.manual_seed(nb + ncols)
    ld = ncols + 6
    L = torch.randn(nb, nb + 4, dtype=torch.float64) * 0.1
    C = torch.randn(nb, ld, dtype=torch.float64)
    L11 = torch.tril(L[:, :nb], -1) + torch.eye(nb, dtype=torch.float64)
    ref = torch.linalg.solve_triangular(L11, C[:, :ncols], upper=False, unitriangular=True)
    Cg, Lg = C.to(cuda), L.to(cuda)
    rc = _native.lib().gelim_gpu_panel_trsm(ptr(Cg), ld, ncols, nb, ptr(Lg), nb + 4, cap, stream_handle(cuda))
    _native.check(rc, "panel_trsm")
    torch.cuda.synchronize()
    assert torch.allclose(Cg.cpu()[:, :ncols], ref, rtol=1e-11, atol=1e-11)
    assert torch.equal(Cg.cpu()[:, ncols:], C[:, ncols:])


def test_big_solver_1024_outer_panels(gelim, cuda):
    """n = 24576: the first order on 1024-column outer panels (plan.hip big_nb;
    K = 1024 trailing updates, profiles/big_nb_lookahead.txt)."""
    n = 24576
    aug = gelim.random_system(n, seed=6, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x = s.solve(aug, check=True)
    s.close()
    ref = torch.linalg.solve(aug[:, :n], aug[:, n].clone())
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-7
    del aug, ref
    torch.cuda.empty_cache()


def test_big_solver_past_old_leaf_cap(gelim, cuda):
    """n = 40000 (12.8 GB): past the round-2 cap of 32768 rows per leaf."""
    n = 40000
    aug = gelim.random_system(n, seed=4, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x = s.solve(aug, check=True)
    s.close()
    ref = torch.linalg.solve(aug[:, :n], aug[:, n].clone())
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-7
    del aug, ref
    torch.cuda.empty_cache()


def _leaf_run(gelim, cuda, P, mode, monkeypatch, streamed):
    from gelim import _native
    from gelim.utils.tensors import ptr, stream_handle

    if streamed:
        monkeypatch.setenv("GELIM_LEAF_STREAM", "1")
    else:
        monkeypatch.delenv("GELIM_LEAF_STREAM", raising=False)
    Pg = P.to(cuda)
    m, ld = P.shape
    ipiv = torch.full((32,), -7, dtype=torch.int32, device=cuda)
    pairs = torch.full((1 + 4 * 32,), -7, dtype=torch.int32, device=cuda)
    info = torch.zeros(4, dtype=torch.int32, device=cuda)
    rc = _native.lib().gelim_gpu_leaf_factor(ptr(Pg), ld, m, 0, mode, ptr(ipiv), ptr(pairs), ptr(info),
                                             stream_handle(cuda))
    _native.check(rc, "leaf_factor")
    torch.cuda.synchronize()
    monkeypatch.delenv("GELIM_LEAF_STREAM", raising=False)
    npairs = int(pairs[0].item())
    return Pg.cpu(), ipiv.cpu(), pairs.cpu()[:1 + 2 * npairs], info.cpu()


@pytest.mark.parametrize("m,kind,mode", [(32, "randn", 1), (1025, "randn", 1), (8192, "randn", 1),
                                         (70000, "randn", 1), (5000, "ties", 1), (3000, "zeros", 0),
                                         (2100, "zeros", 1), (600, "singular", 1)])
def test_streamed_leaf_matches_register_leaf_bitwise(gelim, cuda, monkeypatch, m, kind, mode):
    """The HBM-streamed leaf (leaf_stream.hip, the leaf of panels taller than
    the register file holds) against the register-resident leaf on the same
    panel: identical bits in the factors, ipiv, the net row movement and
    info -- random panels, integer panels full of |a| ties across
    workgroups, panels with exact zeros (the ZERO rule's position keys and
    partial pivoting), and a panel with a zero column (info)."""
    g = torch.Generator().manual_seed(m + mode)
    ld = 34
    if kind == "randn":
        P = torch.randn(m, ld, generator=g, dtype=torch.float64)
    elif kind == "ties":
        P = torch.randint(-3, 4, (m, ld), generator=g).double()
    else:
        P = torch.randn(m, ld, generator=g, dtype=torch.float64)
        P[torch.rand(m, ld, generator=g) < 0.5] = 0.0
        if kind == "singular":
            P[:, 5] = 0.0
    reg = _leaf_run(gelim, cuda, P, mode, monkeypatch, streamed=False)
    st = _leaf_run(gelim, cuda, P, mode, monkeypatch, streamed=True)
    names = ("factors", "ipiv", "pairs", "info")
    for name, a, b in zip(names, reg, st):
        assert torch.equal(a, b), name
    if kind == "singular":
        assert reg[3][0].item() == 6


def test_streamed_leaf_past_register_capacity(gelim, cuda):
    """m = 300000 rows (> 262144, the register leaf's capacity; 82 MB):
    LAPACK's getrf pivots, factors to rounding, the pair list reproduces its
    row order."""
    from gelim import _native

    assert _native.lib().gelim_gpu_leaf_max_rows() >= 540000
    m = 300000
    g = torch.Generator().manual_seed(3)
    P = torch.randn(m, 34, generator=g, dtype=torch.float64)
    from gelim.utils.tensors import ptr, stream_handle

    Pg = P.to(cuda)
    ipiv = torch.zeros(32, dtype=torch.int32, device=cuda)
    pairs = torch.zeros(1 + 4 * 32, dtype=torch.int32, device=cuda)
    info = torch.zeros(4, dtype=torch.int32, device=cuda)
    rc = _native.lib().gelim_gpu_leaf_factor(ptr(Pg), 34, m, 0, 1, ptr(ipiv), ptr(pairs), ptr(info),
                                             stream_handle(cuda))
    _native.check(rc, "leaf_factor")
    torch.cuda.synchronize()
    assert info.cpu()[:2].tolist() == [0, 0]
    lu_, piv_ref = torch.linalg.lu_factor(P[:, :32])
    assert torch.equal(ipiv.cpu().long() + 1, piv_ref.long())
    out = Pg.cpu()
    assert torch.allclose(out[:, :32], lu_, rtol=1e-10, atol=1e-10)
    assert torch.equal(out[:, 32:], P[:, 32:])
    pr = pairs.cpu().tolist()
    moved = {pr[1 + 2 * e]: pr[2 + 2 * e] for e in range(pr[0])}
    perm = list(range(m))
    for j, pj in enumerate(piv_ref.tolist()):
        perm[j], perm[pj - 1] = perm[pj - 1], perm[j]
    assert all(moved.get(d, d) == perm[d] for d in set(moved) | set(range(64)))
    del Pg, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("pivot", ["partial", "zero"])
def test_streamed_leaf_inside_wide_panel_solve(gelim, cuda, monkeypatch, pivot):
    """The whole wide-panel solve with every leaf streamed (GELIM_LEAF_STREAM=1)
    gives the same bits as with the register leaves."""
    n = 3000
    aug = gelim.random_system(n, seed=8, device=cuda) if pivot == "partial" else gelim.synthetic_system(
        n, device=cuda)
    monkeypatch.delenv("GELIM_LEAF_STREAM", raising=False)
    s = gelim.GaussSolver(n, backend="hip", pivot=pivot, device=cuda)
    x0 = s.solve(aug.clone()).cpu()
    s.close()
    monkeypatch.setenv("GELIM_LEAF_STREAM", "1")
    s = gelim.GaussSolver(n, backend="hip", pivot=pivot, device=cuda)
    x1 = s.solve(aug.clone()).cpu()
    s.close()
    assert torch.equal(x0, x1)
