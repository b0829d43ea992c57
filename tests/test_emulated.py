"""In-process emulated communicator: P ranks as threads of
one process on one device, the same collective semantics as the RCCL/gloo
Communicator; plus panel-boundary checkpoint / resume with fault injection
(SURVEY.md §5.3-5.4).  CPU tests here; the GPU variants are in
tests/test_gpu_dist_emulated.py."""
import threading

import pytest
import torch

from gelim.parallel import DistributedGauss, run_emulated
from gelim.parallel.dist_matmul import grid_shape, ring_matmul, summa_matmul
from gelim.utils.checkpoint import InjectedFault


def test_collectives_semantics():
    def body(c):
        r, P = c.rank, c.world_size
        t = torch.full((3,), float(r))
        c.broadcast(t, src=P - 1)
        s = torch.tensor([float(r + 1)])
        c.all_reduce(s)
        m = torch.tensor([float(r)])
        c.all_reduce(m, "max")
        out = torch.empty(2 * P)
        c.all_gather(out, torch.tensor([float(r), float(10 * r)]))
        nxt = torch.empty(1)
        reqs = [c.send(torch.tensor([float(r)]), (r + 1) % P), c.recv(nxt, (r - 1) % P)]
        for q in reqs:
            q.wait()
        c.barrier()
        return t.tolist(), s.item(), m.item(), out.tolist(), nxt.item()

    P = 4
    res = run_emulated(P, body)
    for r, (t, s, m, out, nxt) in enumerate(res):
        assert t == [float(P - 1)] * 3
        assert s == P * (P + 1) / 2 and m == P - 1
        assert out == [v for q in range(P) for v in (float(q), float(10 * q))]
        assert nxt == float((r - 1) % P)


def test_failure_aborts_world():
    def body(c):
        if c.rank == 1:
            raise ValueError("rank 1 failed")
        c.barrier()  # would hang forever without the abort

    with pytest.raises(ValueError, match="rank 1 failed"):
        run_emulated(3, body, timeout_s=30)


@pytest.mark.parametrize("P,n,block", [(1, 100, 16), (2, 130, 16), (3, 257, 8), (4, 200, 32)])
def test_emulated_dist_gauss_cpu(gelim, P, n, block):
    def body(c):
        dg = DistributedGauss(c, n, block=block)
        return dg.solve_(dg.generate_random(seed=17))

    xs = run_emulated(P, body)
    ref = gelim.solve(gelim.random_system(n, seed=17), backend="seq")
    for x in xs:
        assert torch.equal(x, xs[0])
        assert torch.allclose(x, ref, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("P,algo", [(2, "ring"), (4, "ring"), (4, "summa"), (6, "summa")])
def test_emulated_dist_matmul_cpu(P, algo):
    M, K, N = 48, 72, 60
    g = torch.Generator().manual_seed(5)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g)

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

    parts = run_emulated(P, body)
    if algo == "ring":
        C = torch.cat(parts, 0)
    else:
        pr, pc = grid_shape(P)
        C = torch.cat([torch.cat(parts[i * pc:(i + 1) * pc], 1) for i in range(pr)], 0)
    assert torch.allclose(C, A @ B, rtol=1e-4, atol=1e-4)


def _solve_with_ckpt(P, n, block, d, fault=None, resume=False, every=1):
    def body(c):
        dg = DistributedGauss(c, n, block=block)
        loc = dg.generate_random(seed=3)
        ck = dg.checkpointer(d, every=every)
        return dg.solve_(loc, ckpt=ck, resume=resume, fault_at_block=fault)

    return run_emulated(P, body)


@pytest.mark.parametrize("P,every,fault", [(2, 1, 5), (3, 2, 7), (1, 3, 4)])
def test_checkpoint_resume_bitwise(tmp_path, P, every, fault):
    n, block = 180, 16
    clean = _solve_with_ckpt(P, n, block, tmp_path / "clean")
    with pytest.raises(InjectedFault):
        _solve_with_ckpt(P, n, block, tmp_path / "ck", fault=fault, every=every)
    man = (tmp_path / "ck" / "manifest.json").read_text()
    assert f'"block": {(fault - 1) // every * every}' in man
    resumed = _solve_with_ckpt(P, n, block, tmp_path / "ck", resume=True, every=every)
    for a, b in zip(clean, resumed):
        assert torch.equal(a, b)  # same op order after the resume point -> bitwise


def test_checkpoint_mismatch_rejected(tmp_path):
    with pytest.raises(InjectedFault):
        _solve_with_ckpt(2, 120, 16, tmp_path, fault=3)
    with pytest.raises(ValueError, match="ranks"):
        _solve_with_ckpt(3, 120, 16, tmp_path, resume=True)
    with pytest.raises(ValueError, match="does not match"):
        _solve_with_ckpt(2, 120, 8, tmp_path, resume=True)


def test_fault_env_hook(tmp_path, monkeypatch):
    monkeypatch.setenv("GELIM_FAULT_AT_BLOCK", "2")
    monkeypatch.setenv("GELIM_FAULT_RANK", "1")
    with pytest.raises(InjectedFault, match="rank 1"):
        _solve_with_ckpt(2, 100, 16, tmp_path)
    assert threading.active_count() < 50


def test_bench_extras_on_emulated_ranks(gelim):
    """bench.py's strong-scaling sections (distributed Gauss and matmul over
    all ranks) on 2 emulated CPU ranks at reduced sizes: both report, none
    errors."""
    import importlib.util

    from conftest import ROOT

    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def body(c):
        return (bench.bench_dist_gauss(c, gelim, torch, 192), bench.bench_dist_matmul(c, gelim, torch, 64))

    res = run_emulated(2, body)
    for g, m in res:
        assert g["error"] < 1e-9 and g["ranks"] == 2
        assert m["allgather"]["tflops_total"] > 0 and m["ring"]["tflops_total"] > 0
