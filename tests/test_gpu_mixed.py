"""The mixed-precision engine (GaussSolver backend "hip-mixed"): random
butterfly transform + no-pivoting fp32 MFMA LU + fp64 iterative refinement
with an automatic fp64 partial-pivoting fallback (csrc/hip/lu_mixed.hip).

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
    aug = gelim.random_system(n, seed=n + 5, device=cuda)
    s = gelim.GaussSolver(n, backend="hip-mixed", device=cuda)
    x = s.solve(aug, check=True)
    assert s.last_fallback is None, s.last_fallback
    assert s.last_steps <= 4
    ref = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True)
    e_mixed = gelim.ops.gauss.error_metric(x)
    e_fp64 = gelim.ops.gauss.error_metric(ref)
    assert e_mixed <= max(10 * e_fp64, 1e-13), (e_mixed, e_fp64)
    s.close()


def test_mixed_is_selected_by_fp32_dtype(gelim, cuda):
    s = gelim.GaussSolver(300, backend="hip", dtype=torch.float32, device=cuda)
    assert s.backend == "hip-mixed"
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
