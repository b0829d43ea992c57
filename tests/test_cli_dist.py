"""The torchrun launcher CLIs (counterparts of `mpirun -np P ./gauss_*_input`)
on CPU ranks over gloo: output formats of the reference MPI programs and
correct results."""
import os
import re
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(nproc, module, *args, timeout=240):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", module, *args]
    env = dict(os.environ, OMP_NUM_THREADS="1", PYTHONPATH=str(ROOT))
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


def test_dist_gauss_internal_cli():
    out = torchrun(2, "gelim.cli.dist_gauss", "-s", "96", "--block", "16", "--device", "cpu", "--verify")
    assert re.search(r"^Application time: \d+\.\d{6} Secs$", out, re.M), out
    err = float(re.search(r"Max error vs exact solution: (\S+)", out).group(1))
    assert err < 1e-12


def test_dist_gauss_external_cli():
    out = torchrun(3, "gelim.cli.dist_gauss", str(ROOT / "data" / "jpwh_991.coo.npz"), "--block", "32",
                   "--device", "cpu")
    assert re.search(r"^Time:  \d+\.\d{6} seconds$", out, re.M), out
    err = float(re.search(r"^Error: (\S+)$", out, re.M).group(1))
    assert err < 1e-12
    # the MPI program prints these two lines and no header (gauss_mpi/gauss_external_input.c:369-378)
    # (gloo's own connection messages also reach stdout: ignored)
    lines = [ln for ln in out.strip().splitlines() if "Gloo" not in ln and "peer ranks" not in ln]
    assert len(lines) == 2 and lines[0].startswith("Time:  ") and lines[1].startswith("Error: "), out


@pytest.mark.parametrize("algo,nproc", [("ring", 2), ("summa", 4)])
def test_dist_matmul_cli(algo, nproc):
    out = torchrun(nproc, "gelim.cli.dist_matmul", "64", "--algo", algo, "--device", "cpu", "--verify")
    assert re.search(r"^GPU Time: \d+\.\d{6}$", out, re.M), out
    rel = float(re.search(r"Max relative error: (\S+)", out).group(1))
    assert rel < 1e-5


def test_dist_gauss_cli_rbt_internal():
    """--algo rbt: the randomised block-LDU engine over the ranks, same output."""
    out = torchrun(2, "gelim.cli.dist_gauss", "-s", "300", "--algo", "rbt", "--device", "cpu", "--verify")
    assert re.search(r"^Application time: \d+\.\d{6} Secs$", out, re.M), out
    err = float(re.search(r"Max error vs exact solution: (\S+)", out).group(1))
    assert err < 1e-10


def test_dist_gauss_cli_rbt_external():
    out = torchrun(2, "gelim.cli.dist_gauss", str(ROOT / "data" / "jpwh_991.coo.npz"), "--algo", "rbt",
                   "--device", "cpu")
    assert re.search(r"^Time:  \d+\.\d{6} seconds$", out, re.M), out
    err = float(re.search(r"^Error: (\S+)$", out, re.M).group(1))
    assert err < 1e-12
