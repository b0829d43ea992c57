"""Worker bodies for the multi-process tests (spawned by tests/test_dist_cpu.py
and tests/test_gpu_dist.py).  Each worker joins a gloo (CPU) or nccl/RCCL
(GPU) group on 127.0.0.1 and writes its result to a file."""
import os
import sys
import traceback
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def _init(rank, world, port, device, timeout_s=120):
    """device "cpu": gloo CPU ranks; "cuda": every rank on cuda:0 over gloo
    (RCCL refuses two ranks on one GPU) -- device tensors, gloo's
    asynchronous device broadcast / all_reduce, host-staged all_gather."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0" if device == "cuda" else str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from gelim.parallel import comm as C

    if device == "cpu":
        return C.init_from_env(device="cpu", timeout_s=timeout_s)
    return C.init_from_env(backend="gloo", device="cuda:0", timeout_s=timeout_s)


def dead_rank(rank, world, port, outdir):
    """Failure detection: rank 1 dies right after joining; the survivors'
    next collective (the distributed solve's first panel broadcast) must
    raise within the communicator timeout instead of hanging."""
    import time

    from gelim.parallel import DistributedGauss

    comm = _init(rank, world, port, "cpu", timeout_s=15)
    if rank == 1:
        os._exit(3)
    t0 = time.perf_counter()
    try:
        dg = DistributedGauss(comm, 96, block=16)
        dg.solve_(dg.generate_random(seed=1))
        (Path(outdir) / f"ok{rank}.txt").write_text("finished")
    except Exception as e:  # noqa: BLE001
        (Path(outdir) / f"raised{rank}.txt").write_text(f"{time.perf_counter() - t0:.1f} {type(e).__name__}: {e}")
    os._exit(0)


def gauss(rank, world, port, outdir, n, block, seed, device, mode, lookahead=None, tail=None):
    import torch

    import gelim
    from gelim.parallel import DistributedGauss
    from gelim.parallel import comm as C

    try:
        comm = _init(rank, world, port, device)
        dg = DistributedGauss(comm, n, block=block, lookahead=lookahead, tail=tail)
        # G: blocks eliminated as broadcast panels (the rest is the tail system)
        G = dg._panel_blocks(use_tail=bool(dg.lookahead)) if dg.wide else dg.layout.nblocks
        (Path(outdir) / f"meta{rank}.txt").write_text(
            f"{comm.backend} {comm.world_size} {dg.wide} {dg.lookahead} {G}")
        if mode == "random":
            loc = dg.generate_random(seed=seed)
        else:
            aug = gelim.utils.io.load_fixture(mode)
            loc = dg.scatter_from_global(gelim.augment_with_rhs(aug))
        x = dg.solve_(loc)
        torch.save(x.cpu(), Path(outdir) / f"x{rank}.pt")
        C.destroy()
    except Exception:
        (Path(outdir) / f"err{rank}.txt").write_text(traceback.format_exc())
        raise


def matmul(rank, world, port, outdir, M, K, N, algo, device):
    import torch

    from gelim.parallel import comm as C
    from gelim.parallel.dist_matmul import allgather_matmul, grid_shape, ring_matmul, summa_matmul

    try:
        comm = _init(rank, world, port, device)
        g = torch.Generator().manual_seed(5)
        A = torch.randn(M, K, generator=g)
        B = torch.randn(K, N, generator=g)
        dev = comm.device
        if algo in ("ring", "allgather"):
            rows = M // world
            kb = K // world
            fn = ring_matmul if algo == "ring" else allgather_matmul
            C_loc = fn(comm, A[rank * rows:(rank + 1) * rows].to(dev).contiguous(),
                       B[rank * kb:(rank + 1) * kb].to(dev).contiguous())
        else:
            pr, pc = grid_shape(world)
            i, j = divmod(rank, pc)
            mb, ka, kbr, nb = M // pr, K // pc, K // pr, N // pc
            C_loc = summa_matmul(comm, A[i * mb:(i + 1) * mb, j * ka:(j + 1) * ka].to(dev).contiguous(),
                                 B[i * kbr:(i + 1) * kbr, j * nb:(j + 1) * nb].to(dev).contiguous(), (pr, pc))
        torch.save(C_loc.cpu(), Path(outdir) / f"c{rank}.pt")
        C.destroy()
    except Exception:
        (Path(outdir) / f"err{rank}.txt").write_text(traceback.format_exc())
        raise


def rbt(rank, world, port, outdir, n, seed, device, mode, lookahead=True, fast=True):
    """DistributedRBT (randomised block LDU over the ranks): x to x{rank}.pt,
    [steps, berr, fallback] to meta{rank}.txt."""
    import torch

    import gelim
    from gelim.parallel import DistributedRBT
    from gelim.parallel import comm as C

    try:
        comm = _init(rank, world, port, device)
        d = DistributedRBT(comm, n, lookahead=lookahead, single_fast_path=fast)
        if mode == "random":
            loc = d.generate_random(seed=seed)
        else:
            loc = d.scatter_from_global(gelim.augment_with_rhs(gelim.utils.io.load_fixture(mode)))
        x = d.solve_(loc)
        torch.save(x.cpu(), Path(outdir) / f"x{rank}.pt")
        (Path(outdir) / f"meta{rank}.txt").write_text(f"{d.last_steps} {d.last_berr} {d.last_fallback}")
        C.destroy()
    except Exception:
        (Path(outdir) / f"err{rank}.txt").write_text(traceback.format_exc())
        raise
