"""The distributed randomised block-LDU solver (parallel/dist_rbt.py) on CPU
ranks: real gloo processes and emulated ranks, against fp64
torch.linalg.solve.  The CPU ranks run the same schedule, layout and
collectives as the GPU ranks, with torch CPU ops in place of the HIP kernels.

Reference: every MPI worker updates rows at every pivot step
(OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-199)."""
import socket

import pytest
import torch
import torch.multiprocessing as mp

import dist_worker
from gelim.parallel import DistributedRBT, run_emulated
from gelim.parallel.dist_rbt import butterfly_dense, butterfly_diagonals, padded_order


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


def test_padded_order_keeps_butterfly_groups_local():
    for n, P in [(1, 1), (700, 2), (8192, 8), (8193, 8), (5000, 3)]:
        npad = padded_order(n, P)
        assert npad >= n and npad % (512 * P) == 0
        h, nb = npad // 4, npad // 128
        # every column group {j + p h} is in blocks with the same owner
        for j in range(0, h, 128):
            owners = {((j + p * h) // 128) % P for p in range(4)}
            assert len(owners) == 1
        assert (nb // P) * P == nb


def test_dense_butterfly_matches_group_form():
    """The CPU path's dense U matches the kernels' 4 x 4 group form: U is
    block-orthogonal-ish (exactly a product of two scaled butterflies) and
    invertible; U^T A V of the identity is U^T V."""
    ud, vd = butterfly_diagonals(1024)
    U = butterfly_dense(ud, 1024)
    assert torch.linalg.matrix_rank(U).item() == 1024
    # each row has exactly 4 non-zeros (depth-2 butterfly)
    assert int((U != 0).sum(1).max()) == 4


@pytest.mark.parametrize("P,n", [(1, 300), (2, 700), (3, 1000), (4, 1500)])
def test_emulated_dist_rbt_cpu(gelim, P, n):
    def body(c):
        d = DistributedRBT(c, n, single_fast_path=False)
        x = d.solve_(d.generate_random(seed=5))
        return x, d.last_fallback, d.last_berr

    res = run_emulated(P, body, device="cpu", timeout_s=300)
    aug = gelim.random_system(n, seed=5)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    for x, fb, be in res:
        assert fb is None, fb
        assert be <= 4 * torch.finfo(torch.float64).eps
        assert torch.equal(x, res[0][0])
        assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-10


def test_emulated_dist_rbt_singular_falls_back(gelim):
    """A zero column: the no-pivot factorisation cannot succeed, the partial-
    pivoting DistributedGauss takes over and reports the singular matrix."""
    n, P = 400, 2

    def body(c):
        aug = gelim.random_system(n, seed=3)
        aug[:, 57] = 0.0
        d = DistributedRBT(c, n, single_fast_path=False)
        try:
            d.solve_(d.scatter_from_global(aug))
        except gelim.SingularMatrixError:
            return d.last_fallback
        return None

    res = run_emulated(P, body, device="cpu", timeout_s=300)
    assert all(r is not None for r in res)


@pytest.mark.parametrize("world,n", [(2, 900), (3, 1100)])
def test_dist_rbt_processes_cpu(tmp_path, gelim, world, n):
    codes = _spawn(dist_worker.rbt, world, _port(), str(tmp_path), n, 7, "cpu", "random")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0] * world
    xs = [torch.load(tmp_path / f"x{r}.pt") for r in range(world)]
    for x in xs:
        assert torch.equal(x, xs[0])
    aug = gelim.random_system(n, seed=7)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    assert ((xs[0] - ref).abs().max() / ref.abs().max()).item() < 1e-10
    assert (tmp_path / "meta0.txt").read_text().split()[2] == "None"  # no fallback


def test_dist_rbt_reference_matrix_cpu(tmp_path, gelim):
    codes = _spawn(dist_worker.rbt, 2, _port(), str(tmp_path), 991, 0, "cpu", "jpwh_991")
    errs = list(tmp_path.glob("err*.txt"))
    assert not errs, errs[0].read_text()
    assert codes == [0, 0]
    x = torch.load(tmp_path / "x0.pt")
    assert gelim.ops.gauss.error_metric(x) < 1e-12


def test_emulated_dist_rbt_solve_timeout_falls_back_on_every_rank(gelim):
    """One rank's block solves report a timed-out hand-off (its error word
    set): every rank must see it (all_reduce max of the words) and take the
    same partial-pivoting fallback -- not one rank raising while the others
    block in the next collective."""
    n, P = 600, 3

    class Faulty(DistributedRBT):
        def apply(self, rhs):
            out = super().apply(rhs)
            if self.rank == 1 and not getattr(self, "_fired", False):
                self._fired = True
                self._serr.fill_(5)
            return out

    def body(c):
        d = Faulty(c, n, single_fast_path=False)
        x = d.solve_(d.generate_random(seed=9))
        return x, d.last_fallback, int(d._serr.item())

    res = run_emulated(P, body, device="cpu", timeout_s=300)
    aug = gelim.random_system(n, seed=9)
    ref = torch.linalg.solve(aug[:, :n], aug[:, n])
    for x, fb, word in res:
        assert fb == "block-solve hand-off timed out"
        assert word == 0
        assert torch.equal(x, res[0][0])
        assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-10


def test_dist_rbt_pad_warning():
    """n far below the 512 P padding multiple: the flop blow-up is reported."""
    from gelim.parallel.emulated import make_world

    c = make_world(8)[0]
    with pytest.warns(RuntimeWarning, match="padded to 4096"):
        d = DistributedRBT(c, 2048, single_fast_path=False)
    assert d.pad_ratio == 2.0


def test_native_executor_args_layout_matches_python_mirror(gelim):
    """parallel/dist_rbt.py _ExecArgs mirrors csrc/hip/drbt_exec.hip's
    gelim_drbt_args field for field; a drift would hand the executor shifted
    pointers, so size and the offsets of fields late in the block are pinned."""
    import ctypes

    from gelim import _native
    from gelim.parallel.dist_rbt import _ExecArgs

    lay = _native.lib().gelim_drbt_args_layout
    assert lay(0) == ctypes.sizeof(_ExecArgs)
    for which, field in ((1, "Wm"), (2, "side_cap"), (3, "Wfs"), (4, "finfo")):
        assert lay(which) == getattr(_ExecArgs, field).offset, field
