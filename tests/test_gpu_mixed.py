"""The randomised no-pivoting engines (GaussSolver backends "hip-mixed" and
"hip-rbt"): random butterfly transform + no-pivoting MFMA LU (fp32 / fp64
factors, triangular solves of the off-diagonal blocks as GEMMs with the
diagonal blocks' inverses) + fp64 iterative refinement with an automatic fp64
partial-pivoting fallback (csrc/hip/lu_mixed.hip).

Oracles: the exact solution x_i = i + 1 of the random systems, the
reference's fp64 `Error:` values of its .dat matrices and
fp64 torch.linalg.solve.  The reference itself is fp64 only
(OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182); its fp32 run of
the same loop fails saylr4 (error 46.6), which is why refinement + fallback
gate this path."""
import pytest
import torch
from conftest import GOLDEN_ERROR

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 100, 1000, 2048, 4000, 8192])
def test_mixed_random_reaches_fp64(gelim, cuda, n):
    """fp32 trailing products: GMRES-IR gets the fp64 error class back; past
    2048 the fp32 rounding of A21 W can outgrow what 30 GMRES iterations
    repair, and the partial-pivoting fallback answers instead -- always
    correct, never worse than fp64 partial pivoting."""
    aug = gelim.random_system(n, seed=n + 5, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-mixed", device=cuda)
    x = s.solve(aug, check=True)
    if n <= 2048:
        assert s.last_fallback is None, s.last_fallback
        assert s.last_steps <= 6
    ref = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    e_mixed = gelim.ops.gauss.error_metric(x)
    e_fp64 = gelim.ops.gauss.error_metric(ref)
    assert e_mixed <= max(10 * e_fp64, 1e-13), (e_mixed, e_fp64)
    s.close()


def test_mixed_is_explicit_opt_in(gelim, cuda):
    """hip-mixed is slower than hip-rbt at every benched n, so fp32 on the
    blocked backend no longer selects it silently: it must be asked for."""
    with pytest.raises(ValueError, match="hip-mixed"):
        gelim.GaussSolver(300, backend="hip", dtype=torch.float32, device=cuda)
    s = gelim.GaussSolver(300, backend="hip-mixed", device=cuda)
    x, steps = s.solve_refined(gelim.random_system(300, seed=2, device=cuda))
    assert gelim.ops.gauss.error_metric(x) < 1e-9 and steps >= 1


@pytest.mark.parametrize("name", ["jpwh_991", "sherman5", "orsreg_1", "sherman3", "saylr4"])
def test_mixed_reference_matrices(gelim, cuda, name):
    """fp64 error class on the reference's matrices -- by refinement, or by
    the automatic fallback where fp32 cannot get there."""
    A = gelim.utils.io.load_fixture(name)
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    s = gelim.GaussSolver(n, backend="hip-mixed", device=cuda)
    x = s.solve(aug, check=True)
    err = gelim.ops.gauss.error_metric(x)
    assert err <= max(20 * GOLDEN_ERROR[name], 1e-13), (err, s.last_fallback, s.last_steps)
    if name in ("jpwh_991", "sherman5"):
        assert s.last_fallback is None, s.last_fallback


def test_mixed_falls_back_when_fp32_cannot_converge(gelim, cuda):
    """cond(A) = 1e12 >> 1/eps32: the fp32 factors cannot drive the
    refinement, so the fp64 partial-pivoting engine must take over."""
    n = 512
    g = torch.Generator(device=cuda).manual_seed(1)
    Q1, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=cuda, generator=g))
    Q2, _ = torch.linalg.qr(torch.randn(n, n, dtype=torch.float64, device=cuda, generator=g))
    A = (Q1 * torch.logspace(0, -12, n, dtype=torch.float64, device=cuda)) @ Q2
    xt = torch.arange(1, n + 1, dtype=torch.float64, device=cuda)
    aug = torch.zeros(n, n + 8, dtype=torch.float64, device=cuda)
    aug[:, :n] = A
    aug[:, n] = A @ xt
    s = gelim.GaussSolver(n, backend="hip-mixed", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is not None
    ref = torch.linalg.solve(A, aug[:, n])
    # both are fp64 solves of a cond = 1e12 system: they agree to ~cond * eps64
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-3


def test_mixed_singular_raises(gelim, cuda):
    n = 256
    aug = gelim.random_system(n, seed=9, device=cuda)
    aug[:, 17] = 0.0
    s = gelim.GaussSolver(n, backend="hip-mixed", device=cuda)
    with pytest.raises(gelim.SingularMatrixError):
        s.solve(aug, check=True)
    assert s.last_fallback is not None


@pytest.mark.parametrize("tr", ["2", "4", "8"])
@pytest.mark.parametrize("backend", ["hip-mixed", "hip-rbt"])
@pytest.mark.parametrize("n", [130, 1000])
def test_diag_inverses_and_factor(gelim, cuda, backend, n, tr, monkeypatch):
    """Every stored diagonal-block inverse (Gauss-Jordan, fp64; 2 x 8, 4 x 8
    or 8 x 8 tiles on 1024 / 512 / 256 threads, GELIM_GJ_TR) inverts the Schur diagonal
    block the block-LDU factor left in place; fp64 oracle.  (The blocked MFMA
    forms, GELIM_GJ_BLOCKED=1/2, miss this bar by 3-11x on these blocks:
    test_block_inverse_forms_match_torch, profiles/gj_blocked_r4.txt.)"""
    import ctypes

    monkeypatch.setenv("GELIM_GJ_BLOCKED", "0")
    monkeypatch.setenv("GELIM_GJ_TR", tr)

    aug = gelim.random_system(n, seed=3, device=cuda)
    s = gelim.GaussSolver(n, backend=backend, device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    lib = gelim._native.lib()
    ptrs = (ctypes.c_void_p * 3)()
    ldm = int(lib.gelim_mixed_debug_ptrs(s._mixed, ctypes.cast(ptrs, ctypes.c_void_p)))
    np_ = int(lib.gelim_mixed_plan_np(s._mixed))
    dt = torch.float64  # both engines keep the factor in fp64 (hip-mixed: fp32 trailing products)

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


@pytest.mark.parametrize(
    "env", [{}, {"GELIM_RBT_AUX": "1"}, {"GELIM_RBT_LOOKAHEAD": "0"}, {"GELIM_RBT_PAIRS": "0"}])
def test_rbt_schedules_agree(gelim, cuda, env, monkeypatch):
    """The four factorisation schedules -- lookahead over pairs (the default
    from n = 4096), the same with the updates the next inverse does not read
    on a third stream, one-block lookahead, no lookahead; all read when the
    plan is created -- give fp64-class answers on 4200 = 33 blocks (an odd
    count: the pair loop ends on a single block)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = 4200
    aug = gelim.random_system(n, seed=77, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-9
    s.close()


@pytest.mark.parametrize("n", [256, 384, 2048])
def test_rbt_three_stream_small(gelim, cuda, n, monkeypatch):
    """The three-stream schedule forced on small orders (2, 3 and 16 blocks:
    no side update, a panel of one block, the general case)."""
    monkeypatch.setenv("GELIM_RBT_LOOKAHEAD", "1")
    monkeypatch.setenv("GELIM_RBT_AUX", "1")
    aug = gelim.random_system(n, seed=n + 3, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-9
    s.close()


@pytest.mark.parametrize("backend", ["hip-rbt", "hip-mixed"])
def test_not_coresident_falls_back(gelim, cuda, backend, monkeypatch):
    """When the persistent block solves cannot be co-resident (forced here;
    a GPU with fewer CUs, or a busy one), the engine hands the system to the
    partial-pivoting solver instead of failing the solve."""
    monkeypatch.setenv("GELIM_FORCE_NONPERSISTENT", "1")
    n = 700
    aug = gelim.random_system(n, seed=13, device=cuda)
    s = gelim.GaussSolver(n, backend=backend, device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is not None
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-9
    s.close()


@pytest.mark.parametrize("kind", ["dominant", "rbt_like"])
def test_block_inverse_forms_match_torch(gelim, cuda, monkeypatch, kind):
    """gelim_rbt_block_inverse, unblocked (one barrier per pivot; the default)
    and blocked (32- / 16-pivot blocks, MFMA updates: opt-in, measured less
    accurate -- the block updates multiply by the pivot block's inverse), on
    a strided 128 x 128 block, against torch.linalg.inv in fp64; the block
    is read, not written; a zero pivot block is reported through info."""
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
    resid = {}
    for form in ("0", "1", "2"):
        monkeypatch.setenv("GELIM_GJ_BLOCKED", form)
        D = torch.full((128, 128), float("nan"), dtype=torch.float64, device=cuda)
        info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
        blk = bg[30:158, 4:132]
        gelim._native.check(lib.gelim_rbt_block_inverse(ptr(blk), bg.stride(0), 256, ptr(D), ptr(info),
                                                        stream_handle(cuda)), "block_inverse")
        torch.cuda.synchronize()
        assert info.item() == 0x7F7F7F7F
        resid[form] = (D.cpu() @ A - torch.eye(128, dtype=torch.float64)).abs().max().item()
        rel = ((D.cpu() - ref).abs().max() / ref.abs().max()).item()
        bound = 1e-12 * cond * (1 if form == "0" else 1000)
        assert resid[form] < bound and rel < bound, (form, resid[form], rel, cond)
    assert torch.equal(bg.cpu(), big)
    monkeypatch.setenv("GELIM_GJ_BLOCKED", "1")
    Z = torch.zeros(128, 128, dtype=torch.float64, device=cuda)
    D = torch.empty(128, 128, dtype=torch.float64, device=cuda)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(Z), 128, 384, ptr(D), ptr(info), stream_handle(cuda)),
                        "block_inverse")
    torch.cuda.synchronize()
    assert info.item() == 385


@pytest.mark.parametrize("form", ["1", "2"])
@pytest.mark.parametrize("n", [1000, 2048, 4200, 8192])
def test_rbt_with_blocked_inverse(gelim, cuda, monkeypatch, n, form):
    """The whole hip-rbt solve on the blocked MFMA inverse (32- / 16-pivot
    blocks): no fallback, the fp64 error class, a few corrections at most."""
    monkeypatch.setenv("GELIM_GJ_BLOCKED", form)
    aug = gelim.random_system(n, seed=n + 5, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    assert s.last_steps <= 4
    assert gelim.ops.gauss.error_metric(x) < 1e-8
    s.close()


@pytest.mark.parametrize("kind", ["dominant", "rbt_like"])
def test_block_inverse_pairs_bitwise(gelim, cuda, monkeypatch, kind):
    """Two Gauss-Jordan steps per barrier (GELIM_GJ_PAIR=1) perform every
    element's FMAs in the one-step order: the inverse is bit-identical; a
    zero pivot block is reported through info."""
    from gelim.utils.tensors import ptr, stream_handle

    lib = gelim._native.lib()
    g = torch.Generator(device="cpu").manual_seed(11 + len(kind))
    A = torch.randn(128, 128, generator=g, dtype=torch.float64)
    if kind == "dominant":
        A += 64 * torch.eye(128, dtype=torch.float64)
    else:
        Q, _ = torch.linalg.qr(torch.randn(128, 128, generator=g, dtype=torch.float64))
        A = Q @ torch.diag(torch.logspace(0, 4, 128, dtype=torch.float64)) @ Q.T + 0.1 * A
    big = torch.zeros(160, 140, dtype=torch.float64)
    big[7:135, 9:137] = A
    bg = big.to(cuda)
    blk = bg[7:135, 9:137]
    out = {}
    for pair in ("0", "1"):
        monkeypatch.setenv("GELIM_GJ_PAIR", pair)
        D = torch.full((128, 128), float("nan"), dtype=torch.float64, device=cuda)
        info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
        gelim._native.check(lib.gelim_rbt_block_inverse(ptr(blk), bg.stride(0), 0, ptr(D), ptr(info),
                                                        stream_handle(cuda)), "block_inverse")
        torch.cuda.synchronize()
        assert info.item() == 0x7F7F7F7F
        out[pair] = D.cpu()
    assert torch.equal(out["0"], out["1"])
    assert (out["1"] @ A - torch.eye(128, dtype=torch.float64)).abs().max().item() < 1e-12 * torch.linalg.cond(A).item()
    Z = torch.zeros(128, 128, dtype=torch.float64, device=cuda)
    D = torch.empty(128, 128, dtype=torch.float64, device=cuda)
    info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=cuda)
    gelim._native.check(lib.gelim_rbt_block_inverse(ptr(Z), 128, 384, ptr(D), ptr(info), stream_handle(cuda)),
                        "block_inverse")
    torch.cuda.synchronize()
    assert info.item() == 385
