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
    """Every visible GPU: on an 8-GPU node this is P = 8 (the BASELINE
    config's rank count, its padding and super-block sizes)."""
    return torch.cuda.device_count()


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


def test_dist_rbt_8192_graph_over_rccl(tmp_path, gelim):
    """DistributedRBT at the BASELINE size over every GPU, graph-replayed with
    the RCCL broadcasts inside the graph: the third (replayed) solve is
    fp64-class and identical on every rank."""
    world, n = _world(), 8192
    codes = _spawn(dist_worker.rbt_timed, world, _port(), str(tmp_path), n, 47)
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    meta = (tmp_path / "meta0.txt").read_text().split()
    assert meta[0] == "True", meta  # graph replay
    assert meta[3] == "None", meta  # no fallback
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])
    aug = gelim.random_system(n, seed=47)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert _rel(xs[0], ref) < 1e-8


@pytest.mark.parametrize("algo", ["allgather", "ring", "summa"])
def test_dist_matmul_over_rccl(tmp_path, algo):
    """The three distributed matmuls over RCCL against the fp64 product."""
    world = _world()
    M = K = N = 512 * world
    codes = _spawn(dist_worker.matmul, world, _port(), str(tmp_path), M, K, N, algo, "nccl")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    ref = A.double() @ B.double()
    from gelim.parallel.dist_matmul import grid_shape

    if algo == "summa":
        pr, pc = grid_shape(world)
        mb, nb = M // pr, N // pc
        for r in range(world):
            i, j = divmod(r, pc)
            c = torch.load(tmp_path / f"c{r}.pt").double()
            assert _rel(c, ref[i * mb:(i + 1) * mb, j * nb:(j + 1) * nb]) < 1e-5
    else:
        rows = M // world
        for r in range(world):
            c = torch.load(tmp_path / f"c{r}.pt").double()
            assert _rel(c, ref[r * rows:(r + 1) * rows]) < 1e-5


def test_native_rccl_ops_multi(tmp_path):
    """libgelim's RCCL communicator across ranks: broadcasts from every root,
    cross-rank sum / max / min, rank-ordered all_gather, ring send/recv, the
    unique id fetched from the store by ranks != 0."""
    import json

    world = _world()
    codes = _spawn(dist_worker.native_ops_multi, world, _port(), str(tmp_path))
    assert codes == [0] * world
    for r in range(world):
        res = json.loads((tmp_path / f"ops{r}.json").read_text())
        assert res["ok"], res


def test_dead_rank_rccl_raises(tmp_path):
    """The last rank dies after the native communicators exist; the
    survivors' solve raises CommFailure within the watchdog timeout instead
    of hanging in a device wait."""
    world = _world()
    _spawn(dist_worker.dead_rank_rccl, world, _port(), str(tmp_path))
    for r in range(world - 1):
        f = tmp_path / f"raised{r}.txt"
        assert f.exists(), list(tmp_path.iterdir())
        secs, what = f.read_text().split(" ", 1)
        assert float(secs) < 60, what


def test_bench_headline_over_rccl(tmp_path):
    """bench.py --gpus world as a child process (it launches torchrun
    itself): one JSON line, RCCL backend, every GPU joined."""
    import json
    import os
    import subprocess

    world = _world()
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", str(world), "--steps", "3", "--warmup", "1",
                        "--headline-only", "--no-matmul"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["backend"] == "nccl" and line["world_size"] == world and line["n_gpus"] == world
    assert line["max_error"] < 1e-6
