"""The GPU distributed solvers in REAL separate processes: 2-3 ranks sharing
the one MI355X over gloo with device tensors (RCCL refuses two ranks on one
GPU).  gloo's device broadcast is asynchronous and stream-ordered, so the
wide-panel lookahead schedule of DistributedGauss (async panel broadcast into
the double buffer while the previous panel is applied) runs with a truly
asynchronous transport here -- unlike the in-process emulated communicator,
whose broadcast completes before it returns.  Results are compared with the
single-GPU solver and fp64 torch.linalg.solve.

Reference: the MPI master/worker exchange across processes
(OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:136-199)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

import dist_worker

pytestmark = pytest.mark.gpu


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
        p.join(150)
    for p in procs:
        if p.is_alive():
            p.kill()
    return [p.exitcode for p in procs]


def _torch_ref(gelim, aug):
    n = aug.shape[0]
    a = aug.double().cpu()
    return torch.linalg.solve(a[:, :n], a[:, n])


@pytest.mark.parametrize("world,n,block,lookahead", [(2, 1000, 64, True), (2, 2050, 256, True),
                                                     (3, 1530, 128, True), (2, 777, 32, False)])
def test_dist_gauss_gpu_processes(tmp_path, gelim, cuda, world, n, block, lookahead):
    codes = _spawn(dist_worker.gauss, world, _port(), str(tmp_path), n, block, 23, "cuda", "random", lookahead)
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    meta = (tmp_path / "meta0.txt").read_text().split()
    assert meta[:4] == ["gloo", str(world), "True", str(lookahead)]
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])  # replicated solution
    aug = gelim.random_system(n, seed=23, device=cuda)
    single = gelim.GaussSolver(n, backend="hip", device=cuda).solve(aug, check=True).cpu()
    ref = _torch_ref(gelim, aug)
    assert torch.allclose(xs[0], ref, rtol=1e-7, atol=1e-7)
    assert torch.allclose(xs[0], single, rtol=1e-7, atol=1e-7)


@pytest.mark.parametrize("world,n,block,tail", [
    (2, 3000, 128, 0),      # 24 broadcast panels, 12 per rank: every slot of the 3-buffer rotation reused 4x
    (3, 4200, 256, None),   # default 2048-row tail: 9 panels (3 per rank) + the tail engine
    (3, 2500, 64, 0),       # 40 panels, the owner of g+1 changes every step
])
def test_dist_gauss_gpu_processes_many_panels(tmp_path, gelim, cuda, world, n, block, tail):
    """The two-stream lookahead schedule under the truly asynchronous
    transport with G >= 3 P broadcast panels: the NBUF=3 slot rotation
    (ev_rest[g+1-nb] waits), the ev_first cross-stream waits and the side
    stream's applies all run many times (the cases above reach 0-1 panels).
    Checked against the emulated run of the same schedule, the single-GPU
    solver and fp64 torch.linalg.solve."""
    from gelim.parallel import DistributedGauss, run_emulated

    codes = _spawn(dist_worker.gauss, world, _port(), str(tmp_path), n, block, 29, "cuda", "random", True, tail)
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    meta = (tmp_path / "meta0.txt").read_text().split()
    assert meta[:4] == ["gloo", str(world), "True", "True"]
    G = int(meta[4])
    assert G >= 3 * world, f"only {G} broadcast panels"
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])

    def body(c):
        dg = DistributedGauss(c, n, block=block, lookahead=True, tail=tail)
        return dg.solve_(dg.generate_random(seed=29)).cpu()

    emu = run_emulated(world, body, device=cuda, timeout_s=150)[0]
    if world == 2:  # a 2-term sum has one rounding whatever the order: same bits
        assert torch.equal(xs[0], emu)
    else:  # gloo may sum b's 3 partial products in another order: b differs in its
        # last bits, and the solve amplifies that by ~cond(A)
        assert ((xs[0] - emu).abs().max() / emu.abs().max()).item() < 1e-9
    aug = gelim.random_system(n, seed=29, device=cuda)
    ref = _torch_ref(gelim, aug)
    assert torch.allclose(xs[0], ref, rtol=1e-7, atol=1e-7)


def test_dist_gauss_gpu_processes_fixture(tmp_path, gelim, cuda):
    codes = _spawn(dist_worker.gauss, 2, _port(), str(tmp_path), 991, 64, 0, "cuda", "jpwh_991")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0, 0]
    x = torch.load(tmp_path / "x0.pt")
    assert gelim.ops.gauss.error_metric(x) < 1e-12


@pytest.mark.parametrize("world,algo", [(2, "allgather"), (2, "ring"), (4, "summa")])
def test_dist_matmul_gpu_processes(tmp_path, cuda, world, algo):
    M, K, N = 256, 384, 320
    codes = _spawn(dist_worker.matmul, world, _port(), str(tmp_path), M, K, N, algo, "cuda")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g, dtype=torch.float32)
    B = torch.randn(K, N, generator=g, dtype=torch.float32)
    ref = A.double() @ B.double()
    from gelim.parallel.dist_matmul import grid_shape

    if algo == "summa":
        pr, pc = grid_shape(world)
        for r in range(world):
            i, j = divmod(r, pc)
            blk = ref[i * M // pr:(i + 1) * M // pr, j * N // pc:(j + 1) * N // pc]
            c = torch.load(tmp_path / f"c{r}.pt").double()
            assert ((c - blk).abs().max() / blk.abs().max()).item() < 1e-5
    else:
        rows = M // world
        for r in range(world):
            blk = ref[r * rows:(r + 1) * rows]
            c = torch.load(tmp_path / f"c{r}.pt").double()
            assert ((c - blk).abs().max() / blk.abs().max()).item() < 1e-5
