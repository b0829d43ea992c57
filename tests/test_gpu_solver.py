"""GaussSolver on the GPU: accuracy vs torch.linalg.solve (fp64), golden
reference errors on the `.dat` matrices, VERIFY pattern, singular detection,
graph re-use."""
import pytest
import torch

from conftest import GOLDEN_ERROR

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("backend", ["hip", "hip-pivot"])
@pytest.mark.parametrize("n", [1, 2, 7, 64, 300, 1025, 2048, 2500])
def test_random_vs_torch(gelim, cuda, backend, n):
    aug = gelim.random_system(n, seed=n, device=cuda)
    x = gelim.GaussSolver(n, backend=backend, device=cuda).solve(aug, check=True)
    A = aug[:, :n]
    ref = torch.linalg.solve(A, aug[:, n])
    torch.cuda.synchronize()
    assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8 * n)
    assert gelim.ops.gauss.error_metric(x) < 1e-7


@pytest.mark.parametrize("name", list(GOLDEN_ERROR))
@pytest.mark.parametrize("backend", ["hip", "hip-pivot"])
def test_golden_errors_gpu(gelim, cuda, name, backend):
    A = gelim.utils.io.load_fixture(name)
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    x = gelim.GaussSolver(n, backend=backend, device=cuda).solve(aug, check=True)
    err = gelim.ops.gauss.error_metric(x)
    golden = GOLDEN_ERROR[name]
    # different (blocked, FMA) rounding than the reference: same accuracy class
    assert err <= max(20 * golden, 1e-14), (name, err, golden)


@pytest.mark.parametrize("backend,dtype", [("hip", torch.float64), ("hip-pivot", torch.float64),
                                           ("hip-pivot", torch.float32)])
@pytest.mark.parametrize("n", [8, 16, 2048])
def test_internal_verify_pattern_gpu(gelim, cuda, backend, dtype, n):
    aug = gelim.synthetic_system(n, device=cuda, dtype=dtype)
    s = gelim.GaussSolver(n, backend=backend, pivot="zero", dtype=dtype, device=cuda)
    x, bn = s.solve(aug, return_bnorm=True)
    expect = torch.zeros(n, dtype=torch.float64)
    expect[0], expect[-1] = -0.5, 0.5
    eb = torch.full((n,), 0.5, dtype=torch.float64)
    eb[0] = 0.0
    tol = 0 if backend == "hip-pivot" else 1e-12
    assert torch.allclose(x.cpu(), expect, rtol=0, atol=tol)
    assert torch.allclose(bn.cpu(), eb, rtol=0, atol=max(tol, 1e-12))


@pytest.mark.parametrize("backend", ["hip", "hip-pivot"])
def test_singular_detected(gelim, cuda, backend):
    n = 64
    aug = gelim.random_system(n, seed=3, device=cuda)
    aug[:, 10] = aug[:, 3] * 2.0  # rank deficient
    aug[:, 20] = 0.0
    s = gelim.GaussSolver(n, backend=backend, device=cuda)
    s.solve(aug)
    assert s.info() > 0
    with pytest.raises(gelim.SingularMatrixError):
        s.solve(aug, check=True)


def test_graph_replay_and_pointer_change(gelim, cuda):
    n = 500
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    a1 = gelim.random_system(n, seed=1, device=cuda)
    a2 = gelim.random_system(n, seed=2, device=cuda)
    x1 = s.solve(a1).clone()
    x1b = s.solve(a1).clone()  # graph replay
    x2 = s.solve(a2).clone()   # new source pointer -> re-capture
    assert torch.equal(x1, x1b)
    for x, a in ((x1, a1), (x2, a2)):
        assert torch.allclose(x, torch.linalg.solve(a[:, :n], a[:, n]), rtol=1e-9, atol=1e-9)


def test_no_graph_path(gelim, cuda):
    n = 200
    aug = gelim.random_system(n, seed=9, device=cuda)
    xg = gelim.GaussSolver(n, backend="hip", device=cuda, use_graph=True).solve(aug)
    xe = gelim.GaussSolver(n, backend="hip", device=cuda, use_graph=False).solve(aug)
    assert torch.equal(xg, xe)


def test_blocked_ops_composition_gpu(gelim, cuda):
    n = 700
    aug = gelim.random_system(n, seed=5, device=cuda)
    ref = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug)
    x = gelim.blocked_solve_(aug.clone())
    assert torch.allclose(x, ref, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("n", [1500, 2048])
def test_hybrid_matches_pure_fused(gelim, cuda, monkeypatch, n):
    """The hybrid schedule (fused steps, then the resident LU on the trailing
    1024 rows) against the pure fused schedule: same pivots up to rounding."""
    aug = gelim.random_system(n, seed=n + 1, device=cuda)
    x_h = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    monkeypatch.setenv("GELIM_HYBRID", "0")
    x_f = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    torch.cuda.synchronize()
    assert torch.allclose(x_h, x_f, rtol=1e-8, atol=1e-8 * n)
    assert gelim.ops.gauss.error_metric(x_h) < 1e-7


@pytest.mark.parametrize("tail", [512, 640, 768, 896, 1152, 1536])
def test_hybrid_tail_sizes(gelim, cuda, monkeypatch, tail):
    """Every hybrid tail (resident LU in place on the trailing system: 1, 2
    and 4 register slots) against torch.linalg.solve, replayed three times
    (bitwise equal) with info checked each time."""
    n = 2048
    monkeypatch.setenv("GELIM_HYBRID", str(tail))
    aug = gelim.random_system(n, seed=tail, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x = s.solve(aug, check=True).clone()
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8 * n), (x - ref).abs().max().item()
    for _ in range(3):
        assert torch.equal(s.solve(aug, check=True), x)


@pytest.mark.parametrize("n", [1100, 1600, 2048])
def test_resident_schedule_four_slots(gelim, cuda, monkeypatch, n):
    """GELIM_SCHEDULE=resident for 1024 < n <= 2048: the 4-slot resident LU
    (the one variant with register spills) from its own input copy."""
    monkeypatch.setenv("GELIM_SCHEDULE", "resident")
    aug = gelim.random_system(n, seed=n + 5, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x = s.solve(aug, check=True)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8 * n), (x - ref).abs().max().item()
    assert torch.equal(s.solve(aug, check=True), x)


def test_hybrid_tails_interleaved(gelim, cuda, monkeypatch):
    """The round-1 fault scenario: plans with different tails alive at once,
    their graphs replayed interleaved on one stream; every replay bitwise
    equal to the plan's first solve, info clean."""
    n = 2048
    aug = gelim.random_system(n, seed=99, device=cuda)
    plans = []
    for tail in (1024, 896, 768, 640, 512, 1152):
        monkeypatch.setenv("GELIM_HYBRID", str(tail))
        s = gelim.GaussSolver(n, backend="hip", device=cuda)
        plans.append((s, s.solve(aug, check=True).clone()))
    for _ in range(3):
        for s, x in plans:
            assert torch.equal(s.solve(aug, check=True), x)


@pytest.mark.parametrize("zero_col", [100, 1500])
def test_hybrid_singular_column(gelim, cuda, zero_col):
    """A zero column in the fused part (100) or in the resident tail (1500):
    info is the 1-based column of the first zero pivot either way."""
    n = 1600
    aug = gelim.random_system(n, seed=5, device=cuda)
    aug[:, zero_col] = 0.0
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    s.solve(aug)
    assert s.info() == zero_col + 1


@pytest.mark.parametrize("n", [64, 1000, 2048])
def test_fp32_refined_reaches_fp64_accuracy(gelim, cuda, n):
    """fp32 per-pivot elimination on MFMA-free HIP kernels + fp64 residual
    refinement: error lands in the fp64 class, far below plain fp32."""
    aug = gelim.random_system(n, seed=n + 5, device=cuda)
    s32 = gelim.GaussSolver(n, backend="hip-pivot", dtype=torch.float32, device=cuda)
    x32 = s32.solve(aug.float(), check=True)
    x, steps = s32.solve_refined(aug, max_steps=8, check=True)
    torch.cuda.synchronize()
    e32 = gelim.ops.gauss.error_metric(x32)
    e = gelim.ops.gauss.error_metric(x)
    assert steps >= 1
    assert e < 1e-10 and e < e32 / 100, (e32, e, steps)


@pytest.mark.parametrize("name", list(GOLDEN_ERROR))
def test_fp32_refined_golden(gelim, cuda, name):
    A = gelim.utils.io.load_fixture(name)
    n = A.shape[0]
    aug = gelim.augment_with_rhs(A).to(cuda)
    s = gelim.GaussSolver(n, backend="hip-pivot", dtype=torch.float32, device=cuda)
    x32 = s.solve(aug.float(), check=True)
    x, steps = s.solve_refined(aug, max_steps=10, check=True)
    err = gelim.ops.gauss.error_metric(x)
    e32 = gelim.ops.gauss.error_metric(x32)
    # refinement never makes it worse; the well-conditioned matrices reach
    # the fp64 golden class from an fp32 factorisation
    assert err <= e32 * (1 + 1e-6), (name, err, e32)
    if name in ("matrix_10", "jpwh_991"):
        assert err <= max(20 * GOLDEN_ERROR[name], 1e-13), (name, err, steps)


def test_fp64_refined_hip(gelim, cuda):
    n = 1500
    aug = gelim.random_system(n, seed=9, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    x, steps = s.solve_refined(aug, max_steps=2, check=True)
    assert steps >= 1
    assert gelim.ops.gauss.error_metric(x) < 1e-10


@pytest.mark.parametrize("n", [700, 2048, 3000])
def test_forced_nonpersistent_fallback(gelim, cuda, monkeypatch, n):
    """GELIM_FORCE_NONPERSISTENT=1 makes every co-residency check fail: the
    plan must pick the non-persistent schedules (fused steps instead of the
    resident LU / hybrid tail, per-block back substitution launches) and
    still match torch."""
    monkeypatch.setenv("GELIM_FORCE_NONPERSISTENT", "1")
    aug = gelim.random_system(n, seed=n + 17, device=cuda)
    x = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8 * n), (x - ref).abs().max().item()


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-9), (torch.float32, 2e-3)])
@pytest.mark.parametrize("n", [100, 1000])
def test_pivot_plan_resolve(gelim, cuda, dtype, tol, n):
    """hip-pivot keeps its factors: resolve(c) solves A x = c for a NEW
    right-hand side in O(n^2), matching torch (fp32 factors: fp32 accuracy)."""
    aug = gelim.random_system(n, seed=n, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-pivot", dtype=dtype, device=cuda)
    s.solve(aug.to(dtype), check=True)
    A = aug[:, :n]
    for k in range(3):
        c = torch.randn(n, dtype=torch.float64, device=cuda, generator=torch.Generator(cuda).manual_seed(k))
        x = s.resolve(c)
        ref = torch.linalg.solve(A, c)
        assert ((x - ref).abs().max() / ref.abs().max()).item() < tol


def test_refinement_steps_are_quadratic(gelim, cuda):
    """One refinement step (residual + resolve) costs a small fraction of the
    fp32 factorisation it reuses (no re-factoring per step)."""
    import time

    n = 2048
    aug = gelim.random_system(n, seed=3, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-pivot", dtype=torch.float32, device=cuda)
    a32 = aug.to(torch.float32)
    s.solve(a32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    s.solve(a32)
    torch.cuda.synchronize()
    t_factor = time.perf_counter() - t0
    c = aug[:, n].clone()
    s.resolve(c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        s.resolve(c)
    torch.cuda.synchronize()
    t_step = (time.perf_counter() - t0) / 5
    # round 4: the elimination is one persistent launch (13 ms fp32, was 22 ms)
    # while the O(n^2) re-solve's lower triangle is one workgroup: / 5
    assert t_step < t_factor / 5, (t_step, t_factor)
    x, steps = s.solve_refined(aug, max_steps=8)
    assert steps >= 1 and gelim.ops.gauss.error_metric(x) < 1e-9


def zero_rule_position_system(n: int, device, tiny: float = 1e-14):
    """[A | b] on which the internal programs' zero rule (swap only on a zero
    diagonal, first non-zero row BELOW in position order) must track row
    positions: step 0 swaps rows 0 and 5 (column 0 = e5), so at step 1 the
    diagonal (row 1) is zero and the candidates are row 3 (position 3, value
    1) and row 0 (now at position 5, value `tiny`).  The reference takes row 3;
    a rule keyed on the physical row takes row 0 and its 1e-14 pivot ruins the
    solution.  The trailing block is diagonally dominant in the reference's
    final row order, so no further interchange happens."""
    g = torch.Generator().manual_seed(n)
    A = torch.rand(n, n, generator=g, dtype=torch.float64) * 2 - 1
    A[:, 0] = 0.0
    A[5, 0] = 1.0
    A[:, 1] = 0.0
    A[3, 1] = 1.0
    A[0, 1] = tiny
    row_at = list(range(n))  # final position -> row
    row_at[0], row_at[5] = 5, 0
    row_at[1], row_at[3] = 3, 1
    for j in range(2, n):
        A[row_at[j], j] += n
    x = torch.arange(1, n + 1, dtype=torch.float64)
    return torch.cat([A, (A @ x)[:, None]], dim=1).to(device)


def test_zero_rule_position_system_cpu_reference(gelim):
    """The exact reference loop (CPU seq, physical swaps) solves the pattern."""
    aug = zero_rule_position_system(300, "cpu")
    x = gelim.GaussSolver(300, backend="seq", pivot="zero").solve(aug)
    assert gelim.ops.gauss.error_metric(x) < 1e-10


@pytest.mark.parametrize("n", [600, 1500, 2048, 3000])
def test_zero_rule_tracks_positions(gelim, cuda, n):
    """pivot='zero' on every GPU engine (resident LU n <= 1024, fused steps +
    resident tail to 2048, wide-panel leaves above) picks the reference's row
    when an earlier interchange put a lower physical row at a later position."""
    aug = zero_rule_position_system(n, cuda)
    ref = gelim.GaussSolver(n, backend="seq", pivot="zero").solve(aug.cpu())
    for backend in ("hip", "hip-pivot"):
        x = gelim.GaussSolver(n, backend=backend, pivot="zero", device=cuda).solve(aug)
        assert gelim.ops.gauss.error_metric(x) < 1e-9, backend
        assert torch.allclose(x.cpu(), ref, rtol=1e-8, atol=0), backend


@pytest.mark.parametrize("pivot", ["partial", "zero"])
@pytest.mark.parametrize("n", [1, 9, 257, 1000, 2048])
def test_pivot_persistent_matches_two_kernel_form(gelim, cuda, pivot, n, monkeypatch):
    """hip-pivot runs as ONE persistent launch for n <= 2048 (pivot_persist.hip:
    registers hold the matrix, two tagged one-hop exchanges per column); the
    two-kernel-per-column form (forced by GELIM_FORCE_NONPERSISTENT=1) is the
    oracle, together with fp64 torch.linalg.solve."""
    aug = gelim.random_system(n, seed=n + 41, device=cuda)
    if pivot == "zero":  # no interchanges on a random matrix: make it diagonally dominant
        aug[:, :n] += n * torch.eye(n, dtype=torch.float64, device=cuda)
    s1 = gelim.GaussSolver(n, backend="hip-pivot", pivot=pivot, device=cuda)
    x1 = s1.solve(aug, check=True)
    monkeypatch.setenv("GELIM_FORCE_NONPERSISTENT", "1")
    s2 = gelim.GaussSolver(n, backend="hip-pivot", pivot=pivot, device=cuda, use_graph=False)
    x2 = s2.solve(aug, check=True)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    tol = 1e-9
    assert ((x1 - x2).abs().max() / x2.abs().max()).item() < tol
    assert ((x1 - ref).abs().max() / ref.abs().max()).item() < tol
    # the stored factors answer a new right-hand side (resolve) the same way
    c = torch.randn(n, dtype=torch.float64, device=cuda, generator=torch.Generator(cuda).manual_seed(1))
    r1, r2 = s1.resolve(c), s2.resolve(c)
    assert ((r1 - r2).abs().max() / r2.abs().max()).item() < tol
    s1.close()
    s2.close()


@pytest.mark.parametrize("pivot", ["partial", "zero"])
@pytest.mark.parametrize("n", [700, 2048])
def test_graph_replays_bitwise(gelim, cuda, pivot, n):
    """The captured solve replays to the same bits (plan-owned buffers, input
    staged in by an eager copy); fp64 class against torch."""
    aug = gelim.random_system(n, seed=77 + n, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", pivot=pivot, device=cuda)
    xs = [s.solve(aug, check=True).clone() for _ in range(3)]
    assert all(torch.equal(xs[0], x) for x in xs[1:])
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert torch.allclose(xs[0], ref, rtol=1e-8, atol=1e-8 * n)
