"""The distributed algorithms on ONE MI355X through the emulated
communicator (P ranks = P threads): the column block-cyclic
Gauss with its HIP panel / swap+TRSM / fp64 MFMA kernels, and the ring /
SUMMA matmul on the fp32 MFMA kernel, checked against the single-GPU solver
and torch.  RCCL itself refuses two ranks on one device."""
import pytest
import torch

from gelim.parallel import DistributedGauss, run_emulated
from gelim.parallel.dist_matmul import grid_shape, ring_matmul, summa_matmul
from gelim.utils.checkpoint import InjectedFault

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("P,n,block", [(2, 1000, 64), (4, 1537, 32), (8, 2048, 64)])
def test_emulated_dist_gauss_gpu(gelim, cuda, P, n, block):
    def body(c):
        dg = DistributedGauss(c, n, block=block)
        return dg.solve_(dg.generate_random(seed=11))

    xs = run_emulated(P, body, device=cuda, timeout_s=120)
    ref = gelim.solve(gelim.random_system(n, seed=11, device=cuda), backend="hip")
    for x in xs:
        assert x.device.type == "cuda"
        assert torch.equal(x, xs[0])
        assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8)
    assert gelim.ops.gauss.error_metric(xs[0]) < 1e-8


@pytest.mark.parametrize("P,algo", [(4, "ring"), (8, "ring"), (4, "summa"), (8, "summa")])
def test_emulated_dist_matmul_gpu(cuda, P, algo):
    M = K = N = 1024
    g = torch.Generator().manual_seed(2)
    A = torch.randn(M, K, generator=g).to(cuda)
    B = torch.randn(K, N, generator=g).to(cuda)

    def body(c):
        r = c.rank
        if algo == "ring":
            rows, kb = M // P, K // P
            return ring_matmul(c, A[r * rows:(r + 1) * rows].contiguous(), B[r * kb:(r + 1) * kb].contiguous())
        pr, pc = grid_shape(P)
        i, j = divmod(r, pc)
        mb, ka, kbr, nb = M // pr, K // pc, K // pr, N // pc
        return summa_matmul(c, A[i * mb:(i + 1) * mb, j * ka:(j + 1) * ka].contiguous(),
                            B[i * kbr:(i + 1) * kbr, j * nb:(j + 1) * nb].contiguous(), (pr, pc))

    parts = run_emulated(P, body, device=cuda, timeout_s=120)
    if algo == "ring":
        C = torch.cat(parts, 0)
    else:
        pr, pc = grid_shape(P)
        C = torch.cat([torch.cat(parts[i * pc:(i + 1) * pc], 1) for i in range(pr)], 0)
    ref = (A.double() @ B.double())
    assert ((C.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_emulated_checkpoint_resume_gpu(tmp_path, cuda):
    n, block, P = 700, 32, 2

    def run(d, fault=None, resume=False):
        def body(c):
            dg = DistributedGauss(c, n, block=block)
            loc = dg.generate_random(seed=4)
            return dg.solve_(loc, ckpt=dg.checkpointer(d, every=3), resume=resume, fault_at_block=fault)

        return run_emulated(P, body, device=cuda, timeout_s=120)

    clean = run(tmp_path / "a")
    with pytest.raises(InjectedFault):
        run(tmp_path / "b", fault=13)
    resumed = run(tmp_path / "b", resume=True)
    for a, b in zip(clean, resumed):
        assert torch.equal(a, b)


@pytest.mark.parametrize("P,n,block,la", [(1, 3000, 256, True), (1, 3000, 256, False), (3, 2600, 256, True),
                                          (4, 1000, 96, True), (2, 1111, 64, False)])
def test_emulated_dist_gauss_wide(gelim, cuda, P, n, block, la):
    """The GPU distributed path (wide-panel leaves, native panel steps,
    lookahead broadcast) against the single-GPU solver: padded n, partial
    last blocks, with and without lookahead."""
    def body(c):
        dg = DistributedGauss(c, n, block=block, lookahead=la)
        return dg.solve_(dg.generate_random(seed=21))

    xs = run_emulated(P, body, device=cuda, timeout_s=120)
    ref = gelim.solve(gelim.random_system(n, seed=21, device=cuda), backend="hip")
    for x in xs:
        assert x.shape == (n,)
        assert torch.equal(x, xs[0])
        assert torch.allclose(x, ref, rtol=1e-8, atol=1e-8 * n)


def test_emulated_dist_gauss_singular_min_rank(gelim, cuda):
    """Two zero columns owned by different ranks: info reports the FIRST
    one (min over ranks, not max)."""
    n, block, P = 600, 64, 3

    def body(c):
        dg = DistributedGauss(c, n, block=block)
        aug = gelim.random_system(n, seed=8, device=cuda)
        aug[:, 70] = 0.0   # block 1 (rank 1)
        aug[:, 450] = 0.0  # block 7 (rank 1) -- and 130 on rank 2 below
        aug[:, 130] = 0.0  # block 2 (rank 2)
        loc = dg.scatter_from_global(aug)
        dg.factor_(loc)
        return dg.info()

    infos = run_emulated(P, body, device=cuda, timeout_s=120)
    assert infos == [71] * P


@pytest.mark.parametrize("algo", ["allgather", "summa"])
def test_emulated_dist_matmul_16384_8ranks(cuda, algo):
    """BASELINE.json config 5 at full size: 16384^2 fp32 over 8 emulated
    ranks (overlapped allgather and 2-D SUMMA), checked against fp64."""
    from gelim.parallel import allgather_matmul
    from gelim.parallel.dist_matmul import make_summa_groups

    n, P = 16384, 8
    g = torch.Generator(device=cuda).manual_seed(3)
    A = torch.randn(n, n, generator=g, device=cuda)
    B = torch.randn(n, n, generator=g, device=cuda)
    pr, pc = grid_shape(P)

    def body(c):
        r = c.rank
        if algo == "allgather":
            rows = n // P
            return allgather_matmul(c, A[r * rows:(r + 1) * rows], B[r * rows:(r + 1) * rows].contiguous())
        i, j = divmod(r, pc)
        groups = make_summa_groups(c, pr, pc)
        return summa_matmul(c, A[i * n // pr:(i + 1) * n // pr, j * n // pc:(j + 1) * n // pc].contiguous(),
                            B[i * n // pr:(i + 1) * n // pr, j * n // pc:(j + 1) * n // pc].contiguous(), (pr, pc),
                            groups=groups)

    parts = run_emulated(P, body, device=cuda, timeout_s=200)
    if algo == "allgather":
        C = torch.cat(parts, 0)
    else:
        C = torch.cat([torch.cat(parts[i * pc:(i + 1) * pc], 1) for i in range(pr)], 0)
    del parts
    # fp64 reference in row slabs (bounded memory)
    err = 0.0
    for r0 in range(0, n, 2048):
        ref = A[r0:r0 + 2048].double() @ B.double()
        err = max(err, ((C[r0:r0 + 2048].double() - ref).abs().max() / ref.abs().max()).item())
    assert err < 1e-5


def test_emulated_dist_gauss_past_leaf_cap(gelim, cuda):
    """n = 40000 on 2 emulated ranks: every owner panel is taller than the
    round-2 leaf cap (32768 rows); agrees with the single-GPU solver."""
    n, P = 40000, 2

    def body(c):
        dg = DistributedGauss(c, n)
        return dg.solve_(dg.generate_random(seed=31))

    xs = run_emulated(P, body, device=cuda, timeout_s=300)
    aug = gelim.random_system(n, seed=31, device=cuda)
    s = gelim.GaussSolver(n, backend="hip", device=cuda)
    ref = s.solve(aug, check=True)
    s.close()
    del aug
    torch.cuda.empty_cache()
    for x in xs:
        assert torch.equal(x, xs[0])
        assert ((x - ref).abs().max() / ref.abs().max()).item() < 1e-8
