"""The randomised no-pivoting engine (GaussSolver backend "hip-rbt"): random
butterfly transform + no-pivoting fp64 MFMA block LDU (diagonal blocks
inverted by Gauss-Jordan, off-diagonal blocks through GEMMs with the
inverses) + fp64 iterative refinement with an automatic fp64
partial-pivoting fallback (csrc/hip/lu_mixed.hip).  The block triangular
solves of every refinement step run split over the chip
(blk_trsv_split_kernel: K helper workgroups per block row accumulate the
off-diagonal products, the chain workgroup applies the last two blocks).

Oracles: the exact solution x_i = i + 1 of the random systems, the
reference's fp64 `Error:` values of its .dat matrices and
fp64 torch.linalg.solve.  The reference itself is fp64 only
(OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182); its fp32 run of
the same loop fails saylr4 (error 46.6), which is why refinement + fallback
gate this path.  (The fp32-factor engine "hip-mixed" was removed in round 5:
slower than hip-rbt at every n and not convergent at 16384.)"""
import pytest
import torch
from conftest import GOLDEN_ERROR

pytestmark = pytest.mark.gpu


def test_fp32_factor_engine_is_gone(gelim, cuda):
    with pytest.raises(ValueError, match="unknown backend"):
        gelim.GaussSolver(300, backend="hip-mixed", device=cuda)
    with pytest.raises(ValueError, match="hip-pivot"):
        gelim.GaussSolver(300, backend="hip", dtype=torch.float32, device=cuda)
    import numpy as np

    ud = np.ones(2 * 384)
    assert not gelim._native.lib().gelim_mixed_plan_create2(300, ud.ctypes.data, ud.ctypes.data, 0)
    assert "removed" in gelim._native.last_error()


@pytest.mark.parametrize("n", [130, 1000, 3000, 4200])
def test_diag_inverses_and_factor(gelim, cuda, n):
    """Every stored diagonal-block inverse (Gauss-Jordan, fp64, two steps per
    barrier) inverts the Schur diagonal block the block-LDU factor left in
    place -- without lookahead (padded order < 3072) and with the pair
    lookahead on two streams (3000 -> 24 blocks, an even count; 4200 = 33
    blocks: the pair loop ends on a single block); fp64 oracle."""
    import ctypes

    aug = gelim.random_system(n, seed=3, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    lib = gelim._native.lib()
    ptrs = (ctypes.c_void_p * 3)()
    ldm = int(lib.gelim_mixed_debug_ptrs(s._mixed, ctypes.cast(ptrs, ctypes.c_void_p)))
    np_ = int(lib.gelim_mixed_plan_np(s._mixed))
    dt = torch.float64

    def view(addr, count, dtype=dt):
        buf = torch.empty(count, dtype=dtype, device=cuda)
        torch.cuda.synchronize()
        gelim._native.check(lib.gelim_mixed_debug_copy(buf.data_ptr(), addr, count * buf.element_size()), "copy")
        return buf

    M = view(ptrs[0], np_ * ldm).view(np_, ldm)[:, :np_].double()
    D = view(ptrs[1], np_ * 128, torch.float64).view(np_ // 128, 128, 128)
    eye = torch.eye(128, dtype=torch.float64, device=cuda)
    for b in range(np_ // 128):
        blk = M[128 * b:128 * (b + 1), 128 * b:128 * (b + 1)]
        # |D A - I| <= cond(A_bb) eps64-ish: without pivoting a Schur diagonal
        # block of the transformed matrix can reach cond ~1e8
        assert (D[b] @ blk - eye).abs().max().item() < 1e-6, b
    assert gelim.ops.gauss.error_metric(x) < 1e-9
    s.close()


@pytest.mark.parametrize("n", [1, 100, 129, 1000, 2048, 4000, 4200, 5000, 8192])
def test_rbt_random_reaches_fp64(gelim, cuda, n):
    """fp64 block-LDU factors: a few classic refinement steps (each
    contracts the error by ~cond(A_bb) eps64 of the worst diagonal block)."""
    aug = gelim.random_system(n, seed=n + 11, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    assert s.last_steps <= 5
    ref = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    e_rbt = gelim.ops.gauss.error_metric(x)
    e_fp64 = gelim.ops.gauss.error_metric(ref)
    assert e_rbt <= max(10 * e_fp64, 1e-13), (e_rbt, e_fp64)
    s.close()


@pytest.mark.parametrize("name", ["jpwh_991", "sherman5", "orsreg_1", "sherman3", "saylr4"])
def test_rbt_reference_matrices(gelim, cuda, name):
    A = gelim.utils.io.load_fixture(name)
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    err = gelim.ops.gauss.error_metric(x)
    assert err <= max(20 * GOLDEN_ERROR[name], 1e-13), (err, s.last_fallback, s.last_steps)


def test_rbt_ill_conditioned_matches_torch(gelim, cuda):
    """cond(A) = 1e12: fp64 factors still drive the refinement (or the
    fallback takes over); either way x agrees with torch.linalg.solve to
    ~cond * eps64."""
    n = 512
    g = torch.Generator(device=cuda).manual_seed(1)
    Q1, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=cuda, generator=g))
    Q2, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=cuda, generator=g))
    A = (Q1 * torch.logspace(0, -12, n, dtype=torch.float64, device=cuda)) @ Q2
    aug = torch.zeros(n, n + 8, dtype=torch.float64, device=cuda)
    aug[:, :n] = A
    aug[:, n] = A @ torch.arange(1, n + 1, dtype=torch.float64, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    ref = torch.linalg.solve(A, aug[:, n])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-3


def test_rbt_singular_raises(gelim, cuda):
    n = 256
    aug = gelim.random_system(n, seed=9, device=cuda)
    aug[:, 17] = 0.0
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    with pytest.raises(gelim.SingularMatrixError):
        s.solve(aug, check=True)
    assert s.last_fallback is not None


@pytest.mark.parametrize("n", [2048, 8192])
def test_rbt_solves_deterministic(gelim, cuda, n):
    """The split triangular solves add each block row's helper partials in a
    fixed order: the same system gives the same bits every time."""
    aug = gelim.random_system(n, seed=n + 1, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x0 = s.solve(aug).cpu()
    for _ in range(3):
        assert torch.equal(s.solve(aug).cpu(), x0)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n]).cpu()
    assert ((x0 - ref).abs().max() / ref.abs().max()).item() < 1e-9
    s.close()


def test_not_coresident_falls_back(gelim, cuda, monkeypatch):
    """When the persistent block solves cannot be co-resident (forced here;
    a GPU with fewer CUs, or a busy one), the engine hands the system to the
    partial-pivoting solver instead of failing the solve."""
    monkeypatch.setenv("GELIM_FORCE_NONPERSISTENT", "1")
    n = 700
    aug = gelim.random_system(n, seed=13, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is not None
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-9
    s.close()


@pytest.mark.parametrize("kind", ["dominant", "rbt_like"])
def test_block_inverse_matches_torch(gelim, cuda, kind):
    """gelim_rbt_block_inverse on a strided 128 x 128 block against
    torch.linalg.inv in fp64; the block is read, not written; a zero pivot
    block is reported through info."""
    from gelim.utils.tensors import ptr, stream_handle

    lib = gelim._native.lib()
    g = torch.Generator(device="cpu").manual_seed(len(kind))
    A = torch.randn(128, 128, generator=g, dtype=torch.float64)
    if kind == "dominant":
        A += 64 * torch.eye(128, dtype=torch.float64)
    else:  # no small leading minors (what the butterfly transform buys), cond ~1e4
        Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
        A = Q @ torch.diag(torch.logspace(0, 4, 128, dtype=torch.float64)) @ Q.T + 0.1 * A
    ref = torch.linalg.inv(A)
    cond = torch.linalg.cond(A).item()
    big = torch.zeros(200, 134, dtype=torch.float64)
    big[30:158, 4:132] = A
    bg = big.to(cuda)
    D = torch.full((128, 128), float("nan"), dtype=torch.float64, device=cuda)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
    blk = bg[30:158, 4:132]
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(blk), bg.stride(0), 256, ptr(D), ptr(info),
                                                    stream_handle(cuda)), "block_inverse")
    torch.cuda.synchronize()
    assert info.item() == 0x7F7F7F7F
    resid = (D.cpu() @ A - torch.eye(128, dtype=torch.float64)).abs().max().item()
    rel = ((D.cpu() - ref).abs().max() / ref.abs().max()).item()
    assert resid < 1e-12 * cond and rel < 1e-12 * cond, (resid, rel, cond)
    assert torch.equal(bg.cpu(), big)
    Z = torch.zeros(128, 128, dtype=torch.float64, device=cuda)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(Z), 128, 384, ptr(D), ptr(info), stream_handle(cuda)),
                        "block_inverse")
    torch.cuda.synchronize()
    assert info.item() == 385


@pytest.mark.parametrize("logcond", [4, 6])
def test_block_inverse_as_accurate_as_lapack(gelim, cuda, logcond):
    """The Gauss-Jordan inverse of an ill-conditioned (RBT-like: no small
    leading minors) block is as accurate as LAPACK's getrf + getri: the pair
    form without the uniform update's cancellation (round 6; the uniform form
    gave |D A - I| 1.6e-10 against LAPACK's 2.3e-13 at cond 1e4, which cost
    the refinement 4-6 corrections on 1 in 6 random 8192 systems,
    profiles/rbt_seeds_r6.txt).  In place too (the distributed engine's
    slabs)."""
    from gelim.utils.tensors import ptr, stream_handle

    lib = gelim._native.lib()
    g = torch.Generator(device="cpu").manual_seed(11 + logcond)
    Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
    A = Q @ torch.diag(torch.logspace(0, logcond, 128, dtype=torch.float64)) @ Q.T
    A += 10.0 ** (-logcond / 3) * torch.randn(128, 128, generator=g, dtype=torch.float64)
    eye = torch.eye(128, dtype=torch.float64)
    lapack = (torch.linalg.inv(A) @ A - eye).abs().max().item()
    for inplace in (False, True):
        Ag = A.to(cuda)
        D = Ag if inplace else torch.empty_like(Ag)
        info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
        gelim._native.check(lib.gelim_rbt_block_inverse(ptr(Ag), 128, 0, ptr(D), ptr(info), stream_handle(cuda)),
                            "block_inverse")
        torch.cuda.synchronize()
        assert info.item() == 0x7F7F7F7F
        resid = (D.cpu() @ A - eye).abs().max().item()
        assert resid <= 10 * lapack + 1e-14, (logcond, inplace, resid, lapack)


@pytest.mark.parametrize("n", [130, 1000, 4200, 8192])
def test_split_solves_match_one_workgroup_solves(gelim, cuda, n):
    """One apply of the factor (V (LU)^-1 U^T r) through the plan -- split
    triangular solves, K helper workgroups per block row -- against the same
    apply assembled from the one-workgroup-per-block-row kernel
    (gelim_rbt_block_solve, lower then upper) and against dense fp64
    torch.linalg.solve of the same block-triangular systems.  The kernels sum
    the off-diagonal products in different orders, and the factor's diagonal
    blocks reach cond ~1e6 without pivoting, so they agree to rounding times
    that conditioning (3e-8 relative at 8192), not bit for bit: the split
    solve must be as close to the dense reference as the one-workgroup solve
    is (an indexing or hand-off error would be O(1))."""
    import ctypes

    from gelim.utils.tensors import ptr, stream_handle

    lib = gelim._native.lib()
    aug = gelim.random_system(n, seed=n + 17, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    s.solve(aug, check=True)
    plan = s._mixed
    ptrs = (ctypes.c_void_p * 3)()
    ldm = int(lib.gelim_mixed_debug_ptrs(plan, ctypes.cast(ptrs, ctypes.c_void_p)))
    np_ = int(lib.gelim_mixed_plan_np(plan))
    nblk = np_ // 128
    sh = stream_handle(cuda)
    g = torch.Generator(device=cuda).manual_seed(n)
    r = torch.randn(n, dtype=torch.float64, device=cuda, generator=g)
    d_split = torch.empty(n, dtype=torch.float64, device=cuda)
    assert lib.gelim_mixed_apply(plan, ptr(r), 1, ptr(d_split), sh) == 0
    ud = torch.from_numpy(s._ud).to(cuda)
    vd = torch.from_numpy(s._vd).to(cuda)
    c, z, y, x = (torch.empty(np_, dtype=torch.float64, device=cuda) for _ in range(4))
    err = torch.zeros(1, dtype=torch.int32, device=cuda)
    gelim._native.check(lib.gelim_rbt_vec(ptr(r), 1, n, np_, ptr(ud), 1, ptr(c), np_, sh), "rbt_vec")
    gelim._native.check(lib.gelim_rbt_block_solve(ptrs[0], ldm, ptrs[1], nblk, ptr(c), ptr(z), ptr(y), 0, ptr(err),
                                                  sh), "block_solve lower")
    gelim._native.check(lib.gelim_rbt_block_solve(ptrs[0], ldm, ptrs[1], nblk, ptr(y), ptr(x), None, 1, ptr(err),
                                                  sh), "block_solve upper")
    d_old = torch.empty(n, dtype=torch.float64, device=cuda)
    gelim._native.check(lib.gelim_rbt_vec(ptr(x), 1, np_, np_, ptr(vd), 0, ptr(d_old), n, sh), "rbt_vec")
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    # dense reference: forward L_full z = c (block lower part of the factor,
    # its Schur diagonal blocks included), y = Ldiag z, backward U_full x = y
    Mbuf = torch.empty(np_ * ldm, dtype=torch.float64, device=cuda)
    gelim._native.check(lib.gelim_mixed_debug_copy(Mbuf.data_ptr(), ptrs[0], Mbuf.numel() * 8), "copy")
    M = Mbuf.view(np_, ldm)[:, :np_]
    blk = torch.arange(np_, device=cuda) // 128
    lower = blk.view(-1, 1) >= blk.view(1, -1)
    upper = blk.view(-1, 1) <= blk.view(1, -1)
    diag = lower & upper
    zr = torch.linalg.solve(torch.where(lower, M, 0.0), c)
    xr = torch.linalg.solve(torch.where(upper, M, 0.0), torch.where(diag, M, 0.0) @ zr)
    d_ref = torch.empty(n, dtype=torch.float64, device=cuda)
    gelim._native.check(lib.gelim_rbt_vec(ptr(xr), 1, np_, np_, ptr(vd), 0, ptr(d_ref), n, sh), "rbt_vec")
    torch.cuda.synchronize()
    scale = d_ref.abs().max()
    e_split = ((d_split - d_ref).abs().max() / scale).item()
    e_old = ((d_old - d_ref).abs().max() / scale).item()
    assert e_split <= max(4 * e_old, 1e-12), (e_split, e_old)
    assert ((d_split - d_old).abs().max() / scale).item() < 1e-6
    s.close()
