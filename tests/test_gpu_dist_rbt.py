"""The distributed randomised block-LDU solver (parallel/dist_rbt.py) on the
MI355X with its HIP kernels: emulated ranks (P threads sharing the GPU, the
same collectives' semantics), real separate processes over gloo with device
tensors (asynchronous broadcasts: the lookahead's buffer rotation runs under
a truly asynchronous transport), and one rank with and without the
single-GPU fast path.  Oracles: fp64 torch.linalg.solve, the single-GPU
hip-rbt solver and the reference's golden errors.

Reference: OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-199 (every
worker updates rows at every step)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp
from conftest import GOLDEN_ERROR

import dist_worker
from gelim.parallel import DistributedRBT, run_emulated
from gelim.parallel.comm import Communicator

pytestmark = pytest.mark.gpu


def _rel(x, ref):
    return ((x - ref).abs().max() / ref.abs().max()).item()


@pytest.mark.parametrize("P,n,la", [(2, 2000, True), (4, 4000, True), (8, 8192, True), (3, 1400, False)])
def test_emulated_dist_rbt_gpu(gelim, cuda, P, n, la):
    def body(c):
        d = DistributedRBT(c, n, lookahead=la)
        x = d.solve_(d.generate_random(seed=19))
        return x, d.last_fallback, d.last_steps

    res = run_emulated(P, body, device=cuda, timeout_s=240)
    aug = gelim.random_system(n, seed=19, device=cuda)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    single = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    xs = single.solve(aug, check=True)
    single.close()
    for x, fb, steps in res:
        assert fb is None, fb
        assert steps <= 5
        assert torch.equal(x, res[0][0])  # replicated solution, bit-identical
    x = res[0][0]
    assert _rel(x, ref) < 1e-9
    # the same error class as the single-GPU engine (exact solution 1..n)
    assert gelim.ops.gauss.error_metric(x) <= max(10 * gelim.ops.gauss.error_metric(xs), 1e-12)


def test_one_rank_schedule_matches_fast_path(gelim, cuda):
    """One rank: the distributed schedule (lookahead, broadcast buffers,
    super-block solves) and the single-GPU native solve of the same padded
    system agree to the fp64 error class."""
    n = 3000
    c = Communicator(0, 1, cuda, "none")
    out = {}
    for fast in (True, False):
        d = DistributedRBT(c, n, single_fast_path=fast)
        out[fast] = d.solve_(d.generate_random(seed=4))
        assert d.last_fallback is None
        d.close()
    assert _rel(out[False], out[True]) < 1e-11
    assert gelim.ops.gauss.error_metric(out[False]) < 1e-9
    # the fast path is the single-GPU hip-rbt solve (same butterflies): same bits
    aug = gelim.random_system(n, seed=4, device=cuda)
    d = DistributedRBT(c, n)
    s = gelim.GaussSolver(n, backend="hip-rbt", device=cuda)
    assert torch.equal(s.solve(aug), d.solve_(d.scatter_from_global(aug)))
    s.close()
    d.close()


@pytest.mark.parametrize("name", ["jpwh_991", "sherman3", "saylr4"])
def test_emulated_dist_rbt_reference_matrices(gelim, cuda, name):
    A = gelim.utils.io.load_fixture(name)
    aug = gelim.augment_with_rhs(A)

    def body(c):
        d = DistributedRBT(c, A.shape[0])
        return d.solve_(d.scatter_from_global(aug)), d.last_fallback

    res = run_emulated(2, body, device=cuda, timeout_s=240)
    x, fb = res[0]
    assert gelim.ops.gauss.error_metric(x) <= max(20 * GOLDEN_ERROR[name], 1e-13), fb


def test_emulated_dist_rbt_singular_gpu(gelim, cuda):
    n = 1000

    def body(c):
        aug = gelim.random_system(n, seed=2, device=cuda)
        aug[:, 333] = 0.0
        d = DistributedRBT(c, n)
        with pytest.raises(gelim.SingularMatrixError):
            d.solve_(d.scatter_from_global(aug))
        return d.last_fallback

    assert all(r is not None for r in run_emulated(2, body, device=cuda, timeout_s=240))


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
        p.join(200)
    for p in procs:
        if p.is_alive():
            p.kill()
    return [p.exitcode for p in procs]


@pytest.mark.parametrize("world,n", [(2, 3000), (3, 3000)])
def test_dist_rbt_gpu_processes(tmp_path, gelim, cuda, world, n):
    """Real processes sharing the GPU over gloo: 24 / 36 broadcast blocks,
    every buffer slot reused many times under the asynchronous transport."""
    codes = _spawn(dist_worker.rbt, world, _port(), str(tmp_path), n, 23, "cuda", "random")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])
    assert (tmp_path / "meta0.txt").read_text().split()[2] == "None"

    def body(c):
        d = DistributedRBT(c, n)
        return d.solve_(d.generate_random(seed=23)).cpu()

    emu = run_emulated(world, body, device=cuda, timeout_s=200)[0]
    assert _rel(xs[0], emu) < 1e-11
    aug = gelim.random_system(n, seed=23, device=cuda)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n]).cpu()
    assert _rel(xs[0], ref) < 1e-9


@pytest.mark.parametrize("n", [1000, 2048, 4200])
def test_graph_replay_matches_eager(gelim, cuda, n):
    """One rank, no collectives: the factorisation loop and the applies run
    eagerly on the first solve, are captured into hipGraphs on the second and
    replayed from the third -- every solve gives the eager bits."""
    from gelim.parallel import DistributedRBT
    from gelim.parallel.comm import Communicator

    comm = Communicator(0, 1, cuda, "none")
    d = DistributedRBT(comm, n, single_fast_path=False, native_exec=False)  # the Python loop, captured
    assert d.graph
    xs = [d.solve_(d.generate_random(seed=n)).cpu() for _ in range(4)]
    assert set(d._graphs) == {"factor", "apply"} and all(v is not None for v in d._graphs.values())
    dn = DistributedRBT(comm, n, single_fast_path=False)  # the default: native factorisation, captured applies
    assert dn.native_exec
    xs += [dn.solve_(dn.generate_random(seed=n)).cpu() for _ in range(3)]
    assert set(dn._graphs) == {"apply"}
    dn.close()
    e = DistributedRBT(comm, n, single_fast_path=False, graph=False, native_exec=False)
    xe = e.solve_(e.generate_random(seed=n)).cpu()
    for x in xs:
        assert torch.equal(x, xe)
    aug = gelim.random_system(n, seed=n, device=cuda).cpu()
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((xe - ref).abs().max() / ref.abs().max()).item() < 1e-9
    d.close()
    e.close()


@pytest.mark.parametrize("acc", [0, 1])
@pytest.mark.parametrize("M,nblk,K", [(8192, 3, 128), (300, 1, 128), (1000, 8, 256)])
def test_dgemm_block_major(gelim, cuda, acc, M, nblk, K):
    """gelim_gpu_dgemm_bm (dgemm.hip slab_args): B and C as runs of 128-column
    slabs (DistributedRBT's storage) against the fp64 product of the dense
    matrices; bytes outside the touched rows stay as they were."""
    from gelim import _native

    torch.manual_seed(M + nblk + K)
    rows = M + K + 64  # slab height: the operands sit at row offsets inside it
    slabs = torch.randn(nblk, rows, 128, dtype=torch.float64, device=cuda)
    orig = slabs.clone()
    A = torch.randn(M, K, dtype=torch.float64, device=cuda)
    B = slabs[:, 0:K, :]                  # rows [0, K) of every slab
    C = slabs[:, K + 32:K + 32 + M, :]    # rows [K+32, K+32+M) of every slab
    Bd = torch.cat(list(B), dim=1)        # K x 128 nblk
    Cd = torch.cat(list(C), dim=1)
    want = (Cd if acc else 0) - A @ Bd
    _native.check(_native.lib().gelim_gpu_dgemm_bm(C[0].data_ptr(), 128, rows * 128, A.data_ptr(), K, B[0].data_ptr(),
                                                   128, rows * 128, M, 128 * nblk, K, -1.0, acc, 0,
                                                   torch.cuda.current_stream(cuda).cuda_stream), "dgemm_bm")
    torch.cuda.synchronize()
    got = torch.cat(list(slabs[:, K + 32:K + 32 + M, :]), dim=1)
    assert ((got - want).abs().max() / want.abs().max()).item() < 1e-13
    assert torch.equal(slabs[:, :K + 32], orig[:, :K + 32]) and torch.equal(slabs[:, K + 32 + M:], orig[:, K + 32 + M:])


def test_chain_products_match_dgemm(gelim, cuda):
    """drbt_exec.hip's chain kernels (W = Dk B with D -= L W in one launch;
    D -= L W alone) give dgemm.hip's bits, and the fp64 products."""
    from gelim import _native

    lib = _native.lib()
    torch.manual_seed(5)
    Dk, B, L, D0 = (torch.randn(128, 128, dtype=torch.float64, device=cuda) for _ in range(4))
    s = torch.cuda.current_stream(cuda).cuda_stream
    W, D = torch.empty_like(B), D0.clone()
    _native.check(lib.gelim_drbt_chain_products(Dk.data_ptr(), B.data_ptr(), W.data_ptr(), L.data_ptr(), D.data_ptr(),
                                                1, s), "chain_products")
    W2, D2 = torch.empty_like(B), D0.clone()
    _native.check(lib.gelim_gpu_dgemm_ex(W2.data_ptr(), 128, Dk.data_ptr(), 128, B.data_ptr(), 128, 128, 128, 128,
                                         1.0, 0, 0, s), "dgemm W")
    _native.check(lib.gelim_gpu_dgemm_ex(D2.data_ptr(), 128, L.data_ptr(), 128, W2.data_ptr(), 128, 128, 128, 128,
                                         -1.0, 1, 0, s), "dgemm D")
    torch.cuda.synchronize()
    assert torch.equal(W, W2) and torch.equal(D, D2)
    want_w = Dk @ B
    assert ((W - want_w).abs().max() / want_w.abs().max()).item() < 1e-14
    want_d = D0 - L @ want_w
    assert ((D - want_d).abs().max() / want_d.abs().max()).item() < 1e-13
    # the next-row form: D -= L W with W given
    D3, D4 = D0.clone(), D0.clone()
    _native.check(lib.gelim_drbt_chain_products(None, None, W.data_ptr(), L.data_ptr(), D3.data_ptr(), 0, s), "nr")
    _native.check(lib.gelim_gpu_dgemm_ex(D4.data_ptr(), 128, L.data_ptr(), 128, W.data_ptr(), 128, 128, 128, 128,
                                         -1.0, 1, 0, s), "dgemm nr")
    torch.cuda.synchronize()
    assert torch.equal(D3, D4)


def _global_factor(gelim, cuda, P, n, lookahead):
    """The factor of DistributedRBT on P emulated ranks, assembled from the
    ranks' column-block-major slabs into one np x np matrix."""
    def body(c):
        d = DistributedRBT(c, n, lookahead=lookahead, single_fast_path=False, graph=False)
        info = d.factor_(d.generate_random(seed=11))
        torch.cuda.synchronize()
        return d.Mb.cpu(), info

    res = run_emulated(P, body, device=cuda, timeout_s=240)
    npad = res[0][0].shape[1]
    M = torch.empty(npad, npad, dtype=torch.float64)
    for r, (Mb, info) in enumerate(res):
        assert info == 0
        for lb in range(Mb.shape[0]):
            g = lb * P + r
            M[:, g * 128:(g + 1) * 128] = Mb[lb]
    return M


def test_factor_bitwise_across_ranks_and_schedules(gelim, cuda):
    """The split-message lookahead schedule (small [Dinv_k; L_{k+1,k}] message
    on the chain, bulk off it, in-place inverses, no pack) and the one-message
    serial schedule give the SAME factor bits, at P = 1, 2, 4 and 8 (n = 4096
    pads to 4096 for every P, so the system is the same): each element sees the
    same products in the same order whoever updates it."""
    n = 4096
    ref = _global_factor(gelim, cuda, 1, n, False)
    assert torch.isfinite(ref).all()
    for P, la in ((1, True), (2, True), (4, True), (8, True), (4, False)):
        assert torch.equal(_global_factor(gelim, cuda, P, n, la), ref), (P, la)


@pytest.mark.parametrize("n", [2048, 4200])
def test_native_executor_matches_python(gelim, cuda, n):
    """The lookahead factorisation issued natively (csrc/hip/drbt_exec.hip)
    and by the Python loop give the same factor bits and the same solution
    (one rank; the RCCL form is tests/test_gpu_rccl.py)."""
    comm = Communicator(0, 1, cuda, "none")
    out = {}
    for nat in (True, False):
        d = DistributedRBT(comm, n, single_fast_path=False, native_exec=nat, graph=False)
        assert d.native_exec == nat
        loc = d.generate_random(seed=3)
        assert d.factor_(loc) == 0
        torch.cuda.synchronize()
        M = d.Mb.clone()
        x = d.solve_(loc)
        out[nat] = (M, x)
        d.close()
    assert torch.equal(out[True][0], out[False][0])
    assert torch.equal(out[True][1], out[False][1])


@pytest.mark.parametrize("schedule,P", [("native", 4), ("python", 4), ("native", 8)])
def test_one_rank_of_p_replay_runs(tmp_path, schedule, P):
    """scripts/one_rank_of_p.py (rank 1 of a virtual P-rank run, the other
    ranks' chain steps replayed on this GPU) completes and reports times; at
    P = 8 the bulk GEMMs beside the chain run capped (persistent dgemm)."""
    import json
    import os
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    out = tmp_path / "orp.json"
    cmd = [sys.executable, str(root / "scripts" / "one_rank_of_p.py"), "--n", "4096", "--P", str(P), "--rank", "1",
           "--reps", "2", "--json", str(out)] + (["--python-schedule"] if schedule == "python" else [])
    p = subprocess.run(cmd, cwd=root, env=dict(os.environ), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["blocks"] == 32 and res["factor_min_ms"] > 0 and res["apply_min_ms"] > 0
    assert res["schedule"] == ("native executor" if schedule == "native" else "python")
