"""The native CLIs on the GPU."""
import re

import pytest

from conftest import BIN, run_cli

pytestmark = pytest.mark.gpu


def test_internal_default_gpu(cuda):
    r = run_cli(BIN / "gauss_internal_input", "-s", "2048", "--verify", "--json")
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")
    assert lines[1] == "Matrix Size: 2048 ; Threads: 32"
    assert "Backend: hip-blocked" in r.stdout
    assert re.search(r"Application time: \d+\.\d{6} Secs", r.stdout)
    assert "0.00000 -0.50000" in r.stdout and "0.50000 0.50000" in r.stdout


@pytest.mark.parametrize("extra", [["--backend=hip-pivot"], ["--backend=hip-pivot", "--dtype=f32"]])
def test_internal_pivot_gpu(cuda, extra):
    r = run_cli(BIN / "gauss_internal_input", "-s", "256", "--verify", *extra)
    assert r.returncode == 0, r.stderr
    assert "0.00000 -0.50000" in r.stdout


def test_external_gpu(tmp_path, gelim, cuda):
    n, rr, cc, vv = gelim.utils.io.load_coo_npz(gelim.utils.io.fixture_path("sherman3"))
    p = tmp_path / "sherman3.dat"
    gelim.utils.io.write_dat(p, rr, cc, vv, n)
    r = run_cli(BIN / "gauss_external_input", p)
    assert r.returncode == 0, r.stderr
    m = re.search(r"Error: (\S+)", r.stdout)
    assert m and float(m.group(1)) < 1e-11


@pytest.mark.parametrize("name", ["jpwh_991", "sherman3"])
def test_external_rbt_gpu(tmp_path, gelim, cuda, name):
    """hip-rbt on the reference's .dat files: the randomised engine's answer
    (or its automatic partial-pivoting fallback) within 20x of the
    reference's golden fp64 error."""
    from conftest import GOLDEN_ERROR

    n, rr, cc, vv = gelim.utils.io.load_coo_npz(gelim.utils.io.fixture_path(name))
    p = tmp_path / f"{name}.dat"
    gelim.utils.io.write_dat(p, rr, cc, vv, n)
    r = run_cli(BIN / "gauss_external_input", p, "--backend=hip-rbt")
    assert r.returncode == 0, r.stderr
    assert "Backend: hip-rbt" in r.stdout and "hip-rbt: " in r.stdout
    m = re.search(r"Error: (\S+)", r.stdout)
    assert m and float(m.group(1)) <= max(20 * GOLDEN_ERROR[name], 1e-13), r.stdout


def test_internal_rbt_gpu(cuda):
    """The synthetic internal system (exact x = (-0.5, 0, ..., 0, 0.5))."""
    r = run_cli(BIN / "gauss_internal_input", "-s", "1000", "--backend=hip-rbt", "--json")
    assert r.returncode == 0, r.stderr
    m = re.search(r'"max_abs_err": (\S+?)[,}]', r.stdout)
    assert m and float(m.group(1)) < 1e-9, r.stdout
    bad = run_cli(BIN / "gauss_internal_input", "-s", "64", "--backend=hip-rbt", "--verify")
    assert bad.returncode != 0


def test_hip_matmul_cli(cuda):
    r = run_cli(BIN / "hip_matmul", "1024", "--no-seq", "--no-omp", "--verify")
    assert r.returncode == 0, r.stderr
    assert re.search(r"GPU Time: \S+", r.stdout) and "(PASS)" in r.stdout
    for k in ("naive-row", "naive-elem"):
        r = run_cli(BIN / "hip_matmul", "512", f"--kernel={k}", "--no-seq", "--no-omp", "--verify")
        assert r.returncode == 0 and "(PASS)" in r.stdout


def test_hip_matmul_usage():
    r = run_cli(BIN / "hip_matmul")
    assert r.stdout.startswith("Invalid number of arguments: usage")
