"""Multi-process distributed solvers on CPU ranks (gloo over 127.0.0.1):
the same column block-cyclic LU / ring / SUMMA code that runs over RCCL on
GPUs, checked against single-process references."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

import dist_worker


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
        p.join(180)
    for p in procs:
        if p.is_alive():
            p.kill()
    return [p.exitcode for p in procs]


@pytest.mark.parametrize("world,n,block", [(2, 130, 16), (3, 257, 8), (4, 200, 32), (2, 64, 64), (3, 50, 7)])
def test_dist_gauss_random_cpu(tmp_path, gelim, world, n, block):
    codes = _spawn(dist_worker.gauss, world, _port(), str(tmp_path), n, block, 17, "cpu", "random")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    ref = gelim.solve(gelim.random_system(n, seed=17), backend="seq")
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])  # replicated solution, identical on every rank
        assert torch.allclose(x, ref, rtol=1e-9, atol=1e-9)


def test_dist_gauss_reference_matrix_cpu(tmp_path, gelim):
    codes = _spawn(dist_worker.gauss, 2, _port(), str(tmp_path), 991, 32, 0, "cpu", "jpwh_991")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    x = torch.load(tmp_path / "x0.pt")
    assert gelim.ops.gauss.error_metric(x) < 1e-13


@pytest.mark.parametrize("world,algo", [(2, "ring"), (4, "ring"), (3, "ring"), (4, "summa"), (2, "summa"),
                                        (6, "summa"), (2, "allgather"), (3, "allgather"), (4, "allgather")])
def test_dist_matmul_cpu(tmp_path, world, algo):
    M, K, N = 48, 72, 60
    codes = _spawn(dist_worker.matmul, world, _port(), str(tmp_path), M, K, N, algo, "cpu")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)
    ref = A @ B
    parts = [torch.load(tmp_path / f"c{r}.pt") for r in range(world)]
    if algo in ("ring", "allgather"):
        C = torch.cat(parts, 0)
    else:
        from gelim.parallel.dist_matmul import grid_shape

        pr, pc = grid_shape(world)
        C = torch.cat([torch.cat(parts[i * pc:(i + 1) * pc], 1) for i in range(pr)], 0)
    assert torch.allclose(C, ref, rtol=1e-4, atol=1e-4)


def test_column_layout():
    from gelim.parallel import ColumnLayout

    L = ColumnLayout(n=100, P=3, D=16)
    assert L.nblocks == 7 and L.width(6) == 4
    assert L.local_blocks(0) == [0, 3, 6] and L.nloc(0) == 36 and L.nloc(1) == 32
    assert L.first_local_col_after(0, 0) == 16 and L.first_local_col_after(2, 0) == 16
    assert L.first_local_col_after(3, 0) == 32 and L.first_local_col_after(6, 0) == 36
    assert L.first_local_col_after(0, 1) == 0 and L.first_local_col_after(1, 1) == 16


def test_dead_rank_raises_not_hangs(tmp_path):
    """A rank that dies mid-job: the surviving ranks' collectives raise
    (communicator timeout 15 s) instead of blocking forever."""
    codes = _spawn(dist_worker.dead_rank, 3, _port(), str(tmp_path))
    assert codes[1] == 3
    for r in (0, 2):
        f = tmp_path / f"raised{r}.txt"
        assert f.exists(), (codes, list(tmp_path.iterdir()))
        assert float(f.read_text().split()[0]) < 120


def test_dist_handoff_abort_raises(gelim, monkeypatch):
    """A leaf hand-off timeout (info[1] != 0) must fail the solve, never
    back-substitute a half-factored system."""
    from gelim.parallel import DistributedGauss
    from gelim.parallel.comm import Communicator

    dg = DistributedGauss(Communicator(0, 1, torch.device("cpu"), "none"), 64, block=16)
    orig = dg.factor_

    def aborted(loc, *a, **k):
        orig(loc, *a, **k)
        dg._info[1] = 5

    monkeypatch.setattr(dg, "factor_", aborted)
    with pytest.raises(gelim.GelimError, match="code 5"):
        dg.solve_(dg.generate_random(seed=3))


def test_one_rank_process_group_cpu(tmp_path, gelim):
    """force_pg: a one-rank job still creates a (gloo) process group, so every
    collective of the schedule really runs; the solution must equal the plain
    one-rank communicator's bit for bit."""
    from gelim.parallel import DistributedGauss
    from gelim.parallel.comm import Communicator

    codes = _spawn(dist_worker.gauss, 1, _port(), str(tmp_path), 200, 32, 13, "cpu-pg", "random")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0]
    assert (tmp_path / "meta0.txt").read_text().split()[:2] == ["gloo", "1"]
    x = torch.load(tmp_path / "x0.pt")
    dg = DistributedGauss(Communicator(), 200, block=32)
    assert torch.equal(x, dg.solve_(dg.generate_random(seed=13)))
