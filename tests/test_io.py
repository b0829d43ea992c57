"""L1 data / IO: `.dat` reader, fixtures, matrix_gen byte compatibility."""
import numpy as np
import pytest
import torch

from conftest import BIN, REF_DATA, ROOT, have_reference_data, run_cli


def test_matrix_gen_matches_reference_format(tmp_path, gelim):
    out = tmp_path / "m10.dat"
    gelim.utils.io.matrix_gen(10, out)
    text = out.read_text().splitlines()
    assert text[0] == "10 10 100"
    assert text[1] == "1 1 2.000000" and text[2] == "2 1 2.000000"
    assert text[-2] == "10 10 20.000000" and text[-1] == "0 0 0"
    if have_reference_data():
        assert out.read_bytes() == (REF_DATA / "matrix_10.dat").read_bytes()


def test_matrix_gen_cli_bytes(gelim):
    r = run_cli(BIN / "matrix_gen", 10)
    assert r.returncode == 0
    lines = r.stdout.splitlines()
    assert len(lines) == 102
    # column-major walk, value 2*min(row,col)
    assert lines[11] == "1 2 2.000000" and lines[12] == "2 2 4.000000"
    if have_reference_data():
        assert r.stdout.encode() == (REF_DATA / "matrix_10.dat").read_bytes()


def test_matrix_gen_usage():
    r = run_cli(BIN / "matrix_gen")
    assert r.returncode != 0 and "usage" in r.stderr


def test_dat_roundtrip_and_reader(tmp_path, gelim):
    io = gelim.utils.io
    rows = np.array([1, 3, 2, 3], np.int32)
    cols = np.array([1, 1, 2, 3], np.int32)
    vals = np.array([2.5, -1.0, 1e-10, 4.0])
    p = tmp_path / "t.dat"
    io.write_dat(p, rows, cols, vals, 3)
    assert io.dat_size(p) == 3
    A = io.read_dat(p)
    ref = torch.zeros(3, 3, dtype=torch.float64)
    ref[0, 0], ref[2, 0], ref[1, 1], ref[2, 2] = 2.5, -1.0, 1e-10, 4.0
    assert torch.equal(A, ref)
    # padded leading dimension
    A2 = io.read_dat(p, ld=5)
    assert A2.shape == (3, 5) and torch.equal(A2[:, :3], ref) and A2[:, 3:].abs().sum() == 0


def test_dat_reader_errors(tmp_path, gelim):
    with pytest.raises(gelim.GelimError):
        gelim.utils.io.dat_size(tmp_path / "missing.dat")
    bad = tmp_path / "bad.dat"
    bad.write_text("2 2 1\n3 1 1.0\n0 0 0\n")
    with pytest.raises(gelim.GelimError, match="out of range"):
        gelim.utils.io.read_dat(bad)


def test_dat_missing_terminator_ends_at_eof(tmp_path, gelim):
    p = tmp_path / "noterm.dat"
    p.write_text("2 2 2\n1 1 3.0\n2 2 5.0\n")
    A = gelim.utils.io.read_dat(p)
    assert A.tolist() == [[3.0, 0.0], [0.0, 5.0]]


@pytest.mark.parametrize("name", ["matrix_10", "jpwh_991", "sherman3"])
def test_fixtures_match_reference_files(name, gelim):
    io = gelim.utils.io
    F = io.load_fixture(name)
    n = F.shape[0]
    assert F.shape == (n, n)
    if have_reference_data():
        D = io.read_dat(REF_DATA / f"{name}.dat")
        assert torch.equal(F, D)


def test_fixture_header_sizes(gelim):
    sizes = {"matrix_10": 10, "jpwh_991": 991, "orsreg_1": 2205, "sherman5": 3312, "saylr4": 3564,
             "sherman3": 5005, "memplus": 17758}
    for name, n in sizes.items():
        nn, r, c, v = gelim.utils.io.load_coo_npz(gelim.utils.io.fixture_path(name))
        assert nn == n and len(r) == len(c) == len(v) > 0
        assert r.min() >= 1 and r.max() <= n and c.min() >= 1 and c.max() <= n
