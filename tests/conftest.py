"""Test configuration.  `-m "not gpu"` runs everywhere (CPU, gloo);
`-m gpu` needs an MI355X (tests that need a GPU are marked @pytest.mark.gpu)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
REFERENCE = Path("/root/reference")
REF_DATA = REFERENCE / "Pthreads" / "Version-1" / "matrices_dense"
BIN = ROOT / "bin"

# Golden `Error:` values of the reference's own OpenMP external program
# (fp64, SURVEY.md §4.3 / BASELINE.md "Correctness baselines").
GOLDEN_ERROR = {
    "matrix_10": 0.0,
    "jpwh_991": 4.814101e-15,
    "orsreg_1": 2.221803e-10,
    "sherman5": 3.139076e-13,
    "saylr4": 4.203595e-09,
    "sherman3": 4.473903e-13,
}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = ROOT / "gaussian_elimination-cuda-openmp-mpi-pthreads_amd" / "lib" / "libgelim.so"
    if not lib.exists() or not (BIN / "gauss_internal_input").exists():
        subprocess.run([sys.executable, str(ROOT / "__graft_entry__.py"), "build"], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gelim():
    import gelim as g

    return g


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def have_reference_data():
    return REF_DATA.exists()


def run_cli(*args, timeout=600, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    r = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=timeout, env=e)
    return r
