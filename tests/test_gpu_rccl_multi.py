"""The distributed solvers over real RCCL with one rank per GPU (rank r on
cuda:r, libgelim's native communicators, DistributedRBT graph-replayed).
Needs >= 2 visible GPUs: on the one-GPU box every case skips (RCCL refuses
two ranks on one device; the one-rank RCCL group is covered by
tests/test_gpu_rccl.py).  torch.cuda.device_count() does not initialise the
GPU, so the skip test is safe at collection time."""
import multiprocessing as mp
import socket
import sys
from pathlib import Path

import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import dist_worker  # noqa: E402

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one RCCL rank per GPU)")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=fn, args=(r, world) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
    for p in procs:
        if p.is_alive():
            p.kill()
    return [p.exitcode for p in procs]


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max()).item()


def _world():
    return min(torch.cuda.device_count(), 4)


@pytest.mark.parametrize("n", [2048, 4200])
def test_dist_rbt_over_rccl(tmp_path, gelim, n):
    """DistributedRBT with lookahead over RCCL (the distributed schedule, not
    the single-GPU fast path): every rank holds the same solution, fp64-class
    against torch.linalg.solve, no fallback."""
    world = _world()
    codes = _spawn(dist_worker.rbt, world, _port(), str(tmp_path), n, 31, "nccl", "random", True, False)
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])
    assert (tmp_path / "meta0.txt").read_text().split()[2] == "None"
    aug = gelim.random_system(n, seed=31)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert _rel(xs[0], ref) < 1e-9


@pytest.mark.parametrize("lookahead", [False, True])
def test_dist_gauss_over_rccl(tmp_path, gelim, lookahead):
    """DistributedGauss (partial pivoting, column block-cyclic) over RCCL:
    the same x on every rank, equal to the single-GPU solver's to fp64
    rounding (same pivots)."""
    world, n = _world(), 3000
    codes = _spawn(dist_worker.gauss, world, _port(), str(tmp_path), n, 256, 37, "nccl", "random", lookahead)
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    meta = (tmp_path / "meta0.txt").read_text().split()
    assert meta[0] == "nccl" and int(meta[1]) == world
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])
    aug = gelim.random_system(n, seed=37)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert _rel(xs[0], ref) < 1e-7
