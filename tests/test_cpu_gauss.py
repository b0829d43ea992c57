"""CPU reference backends: golden `Error:` values, VERIFY pattern, backend
agreement, pivoting rules, singular detection, CLI output formats."""
import re

import pytest
import torch

from conftest import BIN, GOLDEN_ERROR, REF_DATA, have_reference_data, run_cli

CPU_BACKENDS = ["seq", "omp", "pthreads-v1", "pthreads-v2", "pthreads-v3"]


def _solve_fixture(gelim, name, backend, threads=4):
    A = gelim.utils.io.load_fixture(name)
    aug = gelim.augment_with_rhs(A)
    s = gelim.GaussSolver(A.shape[0], backend=backend, pivot="partial", threads=threads)
    return s.solve(aug)


@pytest.mark.parametrize("backend", CPU_BACKENDS)
def test_golden_jpwh_991_all_backends(gelim, backend):
    x = _solve_fixture(gelim, "jpwh_991", backend)
    err = gelim.ops.gauss.error_metric(x)
    # the reference's exact value: same ops in the same order => same digits
    assert f"{err:e}" == f"{GOLDEN_ERROR['jpwh_991']:e}"


@pytest.mark.parametrize("name", ["matrix_10", "orsreg_1", "sherman5", "saylr4", "sherman3"])
def test_golden_errors_omp(gelim, name):
    x = _solve_fixture(gelim, name, "omp", threads=8)
    err = gelim.ops.gauss.error_metric(x)
    assert f"{err:e}" == f"{GOLDEN_ERROR[name]:e}", (name, err)


def test_backends_bitwise_identical(gelim):
    aug = gelim.random_system(97, seed=3)
    xs = [gelim.GaussSolver(97, backend=b, threads=3).solve(aug) for b in CPU_BACKENDS]
    for x in xs[1:]:
        assert torch.equal(x, xs[0])


@pytest.mark.parametrize("n", [1, 2, 8, 16, 100])
def test_internal_verify_pattern(gelim, n):
    aug = gelim.synthetic_system(n)
    x, bn = gelim.GaussSolver(n, backend="seq", pivot="zero").solve(aug, return_bnorm=True)
    if n == 1:
        assert x.tolist() == [0.0]
        return
    expect = torch.zeros(n, dtype=torch.float64)
    expect[0], expect[-1] = -0.5, 0.5
    assert torch.equal(x, expect)  # exact in fp64
    eb = torch.full((n,), 0.5, dtype=torch.float64)
    eb[0] = 0.0
    assert torch.equal(bn, eb)


def test_zero_pivot_rule_swaps_only_on_zero(gelim):
    # diagonal non-zero but small: ZERO rule keeps it, PARTIAL swaps
    A = torch.tensor([[1e-3, 1.0], [1.0, 1.0]], dtype=torch.float64)
    aug = gelim.augment_with_rhs(A)
    xz = gelim.GaussSolver(2, backend="seq", pivot="zero").solve(aug)
    xp = gelim.GaussSolver(2, backend="seq", pivot="partial").solve(aug)
    assert torch.allclose(xz, torch.tensor([1.0, 2.0], dtype=torch.float64), atol=1e-12)
    assert torch.allclose(xp, torch.tensor([1.0, 2.0], dtype=torch.float64), atol=1e-12)
    # zero diagonal: ZERO rule must swap with the first non-zero row below
    A = torch.tensor([[0.0, 2.0, 1.0], [0.0, 1.0, 3.0], [4.0, 1.0, 1.0]], dtype=torch.float64)
    x = gelim.GaussSolver(3, backend="seq", pivot="zero").solve(gelim.augment_with_rhs(A))
    assert torch.allclose(x, torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64), atol=1e-12)


@pytest.mark.parametrize("backend", CPU_BACKENDS)
def test_singular_raises(gelim, backend):
    A = torch.tensor([[1.0, 2.0], [2.0, 4.0]], dtype=torch.float64)
    with pytest.raises(gelim.SingularMatrixError):
        gelim.GaussSolver(2, backend=backend, threads=2).solve(gelim.augment_with_rhs(A))


def test_v3_many_threads_no_crash(gelim):
    # the reference V3 overflows its thread table for -t > 32
    aug = gelim.random_system(64, seed=5)
    x = gelim.GaussSolver(64, backend="pthreads-v3", threads=48).solve(aug)
    assert gelim.ops.gauss.error_metric(x) < 1e-10


def test_blocked_cpu_matches_reference(gelim):
    aug = gelim.random_system(300, seed=11)
    x_ref = gelim.GaussSolver(300, backend="seq").solve(aug)
    for w in (None, 1, 3, 8, 32):
        x = gelim.blocked_solve_(aug.clone(), width=w)
        assert torch.allclose(x, x_ref, rtol=1e-9, atol=1e-9), w


def test_cpu_panel_factor_matches_lapack(gelim):
    torch.manual_seed(0)
    P = torch.randn(50, 8, dtype=torch.float64)
    lu_, piv_ = torch.linalg.lu_factor(P)
    Q = P.clone()
    piv = torch.zeros(8, dtype=torch.int32)
    info = torch.zeros(4, dtype=torch.int32)
    gelim.ops.lu.panel_factor(Q, piv, info)
    assert torch.equal(piv.long() + 1, piv_[:8].long())  # LAPACK ipiv is 1-based
    assert torch.allclose(Q, lu_, rtol=1e-12, atol=1e-12)
    assert info[0] == 0


# ---- CLIs (CPU backends) ------------------------------------------------------

def test_cli_internal_output_format():
    r = run_cli(BIN / "gauss_internal_input", "-s", "8", "-t", "4", "--backend=seq", "--verify")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert lines[0] == "" and lines[1] == "Matrix Size: 8 ; Threads: 4"
    assert re.fullmatch(r"Application time: \d+\.\d{6} Secs", lines[2])
    assert lines[3] == "0.00000 -0.50000" and lines[10] == "0.50000 0.50000"


def test_cli_internal_v2_v3_headers():
    r = run_cli(BIN / "gauss_internal_input", "-s", "16", "-t", "2", "--backend=pthreads-v2")
    assert "Matrix Size: 16 ; Threads: 2; Block Size: 16" in r.stdout
    r = run_cli(BIN / "gauss_internal_input", "-s", "16", "-t", "2", "--backend=pthreads-v3")
    assert re.search(r"Setting CPU Affinity : (Yes|No)", r.stdout)


def test_cli_internal_help():
    r = run_cli(BIN / "gauss_internal_input", "-h")
    assert r.returncode == 0 and r.stdout.startswith("Usage: ./program -t <num threads> -s <matrix size>")


def test_cli_external_output_and_error(tmp_path, gelim):
    p = tmp_path / "jpwh_991.dat"
    n, rr, cc, vv = gelim.utils.io.load_coo_npz(gelim.utils.io.fixture_path("jpwh_991"))
    if have_reference_data():
        p = REF_DATA / "jpwh_991.dat"
    else:
        gelim.utils.io.write_dat(p, rr, cc, vv, n)
    r = run_cli(BIN / "gauss_external_input", "--backend=omp", p, 4)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert lines[1] == f"Matrix File: {p}; Matrix Size: 991 ; Threads: 4"
    assert re.fullmatch(r"Time:  \d+\.\d{6} seconds", lines[2])
    assert lines[3] == "Error: 4.814101e-15"


def test_cli_external_usage_and_missing_file(tmp_path):
    r = run_cli(BIN / "gauss_external_input")
    assert r.returncode != 0 and "usage:" in r.stderr
    r = run_cli(BIN / "gauss_external_input", "--backend=seq", tmp_path / "nope.dat")
    assert r.returncode != 0 and "The matrix file open error" in r.stderr


def test_refinement_cpu_seq(gelim):
    """Iterative refinement on a CPU backend: fp64 elimination + fp64
    residual corrections never make the solution worse, and converge."""
    import torch
    n = 96
    aug = gelim.random_system(n, seed=11)
    s = gelim.GaussSolver(n, backend="seq")
    x0 = s.solve(aug)
    x, steps = s.solve_refined(aug, max_steps=3)
    assert 0 <= steps <= 3
    e0 = gelim.ops.gauss.error_metric(x0)
    e1 = gelim.ops.gauss.error_metric(x)
    assert e1 <= max(e0, 1e-14)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert torch.allclose(x, ref, rtol=1e-12, atol=1e-12)


def test_cli_gpu_backend_without_gpu_says_so():
    """A GPU backend on a GPU-less host names the problem and the CPU
    alternative instead of a runtime error from inside a plan."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    r = run_cli(BIN / "gauss_internal_input", "-s", "32")
    assert r.returncode != 0
    assert "no HIP device found" in r.stderr and "--backend=omp" in r.stderr
