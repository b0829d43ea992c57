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
    asynchronous device broadcast / all_reduce, host-staged all_gather;
    "nccl": RCCL, rank r on cuda:r (the process group is created even for
    one rank)."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0" if device == "cuda" else str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from gelim.parallel import comm as C

    if device == "cpu":
        return C.init_from_env(device="cpu", timeout_s=timeout_s)
    if device == "cpu-pg":  # gloo group even for one rank (force_pg)
        return C.init_from_env(device="cpu", timeout_s=timeout_s, force_pg=True)
    if device == "nccl":  # RCCL: one rank per GPU (a one-rank group on the one-GPU box)
        return C.init_from_env(backend="nccl", device=f"cuda:{rank}", timeout_s=timeout_s, force_pg=True)
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


def rccl_one_rank(outdir, n_gauss=2048, n_rbt=2048):
    """Every distributed schedule through a ONE-rank RCCL process group on
    cuda:0, each result next to the same schedule on the plain one-rank
    communicator (backend "none": no collective runs).  One rank's
    collectives leave the data as it is, so the two must agree bit for bit;
    what differs is that every broadcast / all_gather / all_reduce is a real
    RCCL call on the communicator's stream, ordered by events against the
    main and side streams.  Writes res.json and the solutions."""
    import json
    import time

    import torch
    import torch.distributed as dist

    import gelim
    from gelim.parallel import DistributedGauss, DistributedRBT
    from gelim.parallel import comm as C
    from gelim.parallel.dist_matmul import allgather_matmul, make_summa_groups, summa_matmul
    from gelim.utils.tensors import side_stream, side_stream_stats

    out = Path(outdir)
    res = {}
    try:
        comm = _init(0, 1, 0, "nccl")
        dev = comm.device
        none = C.Communicator(0, 1, dev, "none")
        res.update(backend=comm.backend, pg=comm.pg, initialized=dist.is_initialized(),
                   pg_backend=str(dist.get_backend()), world=dist.get_world_size())
        side = side_stream(dev)
        res["native"] = comm.native
        res["overlap_own_stream"] = comm.overlap_probe(side)
        os.environ["GELIM_COMM"] = "torch"  # torch.distributed's RCCL path (same dedicated stream)
        res["overlap_torch_stream"] = comm.overlap_probe(side)
        os.environ.pop("GELIM_COMM")
        res["streams"] = {"side": side.cuda_stream, "comm": comm.comm_stream().cuda_stream,
                          "default": torch.cuda.current_stream(dev).cuda_stream}
        res["side_stream_stats"] = list(side_stream_stats())

        def run_gauss(c, n, **kw):
            dg = DistributedGauss(c, n, **kw)
            x = dg.solve_(dg.generate_random(seed=41))
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            x = dg.solve_(dg.generate_random(seed=41))
            torch.cuda.synchronize(dev)
            return x.cpu(), time.perf_counter() - t0, dg._panel_blocks(use_tail=bool(dg.lookahead))

        for tag, kw in (("gauss_la_tail0", dict(tail=0)), ("gauss_la", {}), ("gauss_serial", dict(lookahead=False))):
            xp, tp, G = run_gauss(comm, n_gauss, **kw)
            xn, tn, _ = run_gauss(none, n_gauss, **kw)
            os.environ["GELIM_COMM"] = "torch"
            xt, tt, _ = run_gauss(comm, n_gauss, **kw)
            os.environ.pop("GELIM_COMM")
            torch.save(xp, out / f"{tag}.pt")
            res[tag] = {"bitwise": bool(torch.equal(xp, xn)), "torch_path_bitwise": bool(torch.equal(xt, xn)),
                        "panels": G, "rccl_s": tp, "none_s": tn, "rccl_torch_path_s": tt}

        def run_rbt(c, n, graph=True):
            """Three solves: eager, captured + replayed, replayed (graph=True)."""
            d = DistributedRBT(c, n, single_fast_path=False, graph=graph)
            xs = []
            for _ in range(3):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                xs.append(d.solve_(d.generate_random(seed=43)).cpu())
                torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            meta = (d.last_steps, d.last_berr, d.last_fallback, d.graph)
            d.close()
            return xs, dt, meta

        xp, tp, mp_ = run_rbt(comm, n_rbt)
        xn, tn, mn_ = run_rbt(none, n_rbt)
        xe, te, _ = run_rbt(comm, n_rbt, graph=False)
        os.environ["GELIM_COMM"] = "torch"
        xt, tt, mt_ = run_rbt(comm, n_rbt)  # torch.distributed's RCCL: eager (no capture)
        os.environ.pop("GELIM_COMM")
        xe = xe + xt
        torch.save(xp[-1], out / "rbt.pt")
        res["rbt"] = {"bitwise": bool(torch.equal(xp[-1], xn[-1])), "rccl_s": tp, "none_s": tn, "rccl_eager_s": te,
                      "rccl_torch_path_s": tt, "graph_torch_path": mt_[3],
                      "graph_rccl": mp_[3], "graph_none": mn_[3],
                      "replay_equals_eager": all(torch.equal(x, xe[0]) for x in xp + xn + xe),
                      "steps": mp_[0], "berr": mp_[1], "fallback": mp_[2]}
        d1 = DistributedRBT(none, n_rbt)  # the single-GPU native engine on the same system
        d1.solve_(d1.generate_random(seed=43))
        res["rbt"]["native_steps"], res["rbt"]["native_berr"] = d1.last_steps, d1.last_berr
        d1.close()

        g = torch.Generator(device=dev).manual_seed(3)
        A = torch.randn(512, 768, generator=g, device=dev)
        B = torch.randn(768, 640, generator=g, device=dev)
        ref = A @ B
        cp = allgather_matmul(comm, A, B)
        cn = allgather_matmul(none, A, B)
        res["matmul_allgather"] = {"bitwise": bool(torch.equal(cp, cn)),
                                   "rel": float(((cp.double() - ref.double()).abs().max() / ref.abs().max()).item())}
        groups = make_summa_groups(comm, 1, 1)
        sp = summa_matmul(comm, A, B, (1, 1), groups=groups, panels=3)
        sn = summa_matmul(none, A, B, (1, 1), panels=3)
        res["matmul_summa"] = {"bitwise": bool(torch.equal(sp, sn)),
                               "subgroup_backend": groups[0].backend, "subgroup_pg": groups[0].pg}
        # libgelim's RCCL communicator directly: every collective x every dtype
        nc = comm.rccl()
        cur = torch.cuda.current_stream(dev).cuda_stream
        native = {}
        for dt in (torch.float64, torch.float32, torch.int32, torch.int64, torch.uint8):
            base = (torch.arange(1, 301, device=dev) % 100).to(dt)
            t = base.clone()
            nc.bcast(t, 0, cur)
            native[f"bcast_{dt}"] = bool(torch.equal(t, base))
            for op in ("sum", "max", "min"):
                t = base.clone()
                nc.allreduce(t, op, cur)
                native[f"allreduce_{op}_{dt}"] = bool(torch.equal(t, base))
            o = torch.zeros(300, dtype=dt, device=dev)
            nc.allgather(o, base, cur)
            native[f"allgather_{dt}"] = bool(torch.equal(o, base))
            o = torch.zeros(300, dtype=dt, device=dev)
            nc.sendrecv(base, 0, o, 0, cur)
            native[f"sendrecv_{dt}"] = bool(torch.equal(o, base))
        torch.cuda.synchronize(dev)
        res["native_ops"] = native
        # point-to-point through RCCL: a batched send to / receive from the rank itself
        t = torch.arange(1000, dtype=torch.float64, device=dev)
        r = torch.zeros_like(t)
        try:
            for q in comm.sendrecv(t, 0, r, 0):
                q.wait()
            torch.cuda.synchronize(dev)
            res["p2p_self"] = {"ok": bool(torch.equal(t, r))}
        except Exception as e:  # noqa: BLE001
            res["p2p_self"] = {"ok": False, "error": repr(e)[:300]}
        comm.barrier()
        C.destroy()
        res["ok"] = True
    except Exception:
        res["ok"] = False
        res["traceback"] = traceback.format_exc()
    (out / "res.json").write_text(json.dumps(res, indent=1, default=str))
    if not res["ok"]:
        raise SystemExit(1)


def rccl_watchdog(outdir):
    """Failure detection on the native RCCL path, on ONE GPU:
    a one-rank native broadcast queued behind a bounded 2 s spin kernel
    stands in for a collective whose peer never arrives.  With the watchdog
    at timeout 0.5 s:
      wait_point  the guarded host wait (Communicator.synchronize, the
                  solvers' wait points) raises CommFailure after ~0.5 s;
      async       with the main thread in plain Python (no wait point), the
                  watchdog thread raises CommFailure in it asynchronously.
    Both times every native communicator is aborted (ncclCommAbort) and a
    further collective raises at once.  A one-rank in-place broadcast
    queues no RCCL kernel, so the abort has no device work to cancel; the
    spin kernel ends on its own and the process exits normally."""
    import json
    import time

    import torch

    from gelim import _native
    from gelim.parallel import comm as C
    from gelim.utils.tensors import ptr

    out = Path(outdir)
    res = {}
    try:
        comm = _init(0, 1, 0, "nccl", timeout_s=120)
        dev = comm.device
        res["native"] = comm.native
        lib = _native.lib()
        t = torch.zeros(4096, dtype=torch.float64, device=dev)
        words = torch.zeros(2, dtype=torch.int32, device=dev)
        spin_ticks = 200_000_000  # 2 s of s_memrealtime (100 MHz)

        steps = {}

        def stall_then_bcast():
            a = time.perf_counter()
            comm.broadcast(t, 0)  # creates the communicator (and the watchdog)
            steps["create_bcast"] = time.perf_counter() - a
            comm.synchronize()
            # the communicator stream exists before the stall: creating it
            # probes it against the default stream, which would wait for the
            # spin kernel (utils/tensors.dedicated_stream)
            comm.comm_stream()
            steps["sync"] = time.perf_counter() - a
            C.start_watchdog(timeout_s=0.5, poll_s=0.02)
            words.zero_()
            steps["zero"] = time.perf_counter() - a
            _native.check(lib.gelim_gpu_probe_kernel(torch.cuda.current_stream(dev).cuda_stream, ptr(words), 0,
                                                     spin_ticks), "probe_kernel")
            steps["spin_launch"] = time.perf_counter() - a
            h = comm.broadcast_async(t, 0)
            steps["bcast_async"] = time.perf_counter() - a
            return h

        # 1. the guarded wait point
        ts = time.perf_counter()
        h = stall_then_bcast()
        t0 = time.perf_counter()
        probe = torch.cuda.Event()
        probe.record(torch.cuda.current_stream(dev))
        diag = {"issue_s": t0 - ts, "steps": dict(steps), "stream_busy_after_issue": not probe.query(), "pending": len(C.watchdog()._pending),
                "timeout_s": C.watchdog().timeout_s}
        try:
            h.wait()
            comm.synchronize()
            res["wait_point"] = {"raised": False, "sync_s": time.perf_counter() - t0, **diag}
        except C.CommFailure as e:
            res["wait_point"] = {"raised": True, "after_s": time.perf_counter() - t0, "msg": str(e)[:200],
                                 "native_left": len(C._NATIVE)}
        try:
            comm.broadcast(t, 0)
            res["wait_point"]["later_call_raised"] = False
        except C.CommFailure:
            res["wait_point"]["later_call_raised"] = True
        torch.cuda.synchronize(dev)  # the spin kernel ends by itself
        time.sleep(0.2)
        res["wait_point"]["native_left_later"] = len(C._NATIVE)  # the watchdog thread aborted them
        # fresh communicator + watchdog for the second case
        wd = C.watchdog()
        wd.stop()
        C._WATCHDOG.clear()
        comm._rccl = None
        comm.key = "world-2"

        # 2. no wait point: the watchdog thread raises in the main thread
        h = stall_then_bcast()
        t0 = time.perf_counter()
        try:
            for _ in range(500):  # 5 s of plain Python
                time.sleep(0.01)
            res["async"] = {"raised": False}
        except C.CommFailure:
            res["async"] = {"raised": True, "after_s": time.perf_counter() - t0}
        torch.cuda.synchronize(dev)
        time.sleep(0.2)
        res["async"]["native_left_later"] = len(C._NATIVE)
        C.destroy(abort=True)
        res["ok"] = True
    except Exception:
        res["ok"] = False
        res["traceback"] = traceback.format_exc()
    (out / "res.json").write_text(json.dumps(res, indent=1, default=str))


def dead_rank_rccl(rank, world, port, outdir):
    """dead_rank over RCCL with libgelim's native communicators (one rank per
    GPU): the last rank dies after the communicator exists; the survivors'
    distributed solve must raise CommFailure within the watchdog timeout
    (not hang in a device wait)."""
    import time

    import torch

    from gelim.parallel import DistributedGauss
    from gelim.parallel import comm as C

    comm = _init(rank, world, port, "nccl", timeout_s=120)
    C.start_watchdog(timeout_s=5.0, poll_s=0.05)
    t = torch.ones(1024, dtype=torch.float64, device=comm.device)
    comm.all_reduce(t)  # every rank's native communicator exists
    comm.synchronize()
    if rank == world - 1:
        os._exit(3)
    t0 = time.perf_counter()
    try:
        dg = DistributedGauss(comm, 4096, block=256)
        dg.solve_(dg.generate_random(seed=1))
        (Path(outdir) / f"ok{rank}.txt").write_text("finished")
    except Exception as e:  # noqa: BLE001
        (Path(outdir) / f"raised{rank}.txt").write_text(f"{time.perf_counter() - t0:.1f} {type(e).__name__}: {e}")
    os._exit(0)


def native_ops_multi(rank, world, port, outdir):
    """libgelim's RCCL communicator across ranks (one per GPU): broadcasts
    from every root, cross-rank sum / max / min, a rank-ordered all_gather
    and a ring send/recv, each checked against its closed form; results to
    ops{rank}.json."""
    import json

    import torch

    from gelim.parallel import comm as C

    res = {}
    try:
        comm = _init(rank, world, port, "nccl")
        dev = comm.device
        nc = comm.rccl()
        cur = torch.cuda.current_stream(dev).cuda_stream
        for dt in (torch.float64, torch.float32, torch.int32, torch.int64):
            base = torch.arange(1, 257, device=dev).to(dt)
            for root in range(world):
                t = base * (rank + 1)
                nc.bcast(t, root, cur)
                res[f"bcast_root{root}_{dt}"] = bool(torch.equal(t, base * (root + 1)))
            for op, want in (("sum", base * (world * (world + 1) // 2)), ("max", base * world), ("min", base)):
                t = base * (rank + 1)
                nc.allreduce(t, op, cur)
                res[f"allreduce_{op}_{dt}"] = bool(torch.equal(t, want))
            o = torch.zeros(256 * world, dtype=dt, device=dev)
            nc.allgather(o, base * (rank + 1), cur)
            want = torch.cat([base * (q + 1) for q in range(world)])
            res[f"allgather_{dt}"] = bool(torch.equal(o, want))
            o = torch.zeros(256, dtype=dt, device=dev)
            nc.sendrecv(base * (rank + 1), (rank + 1) % world, o, (rank - 1) % world, cur)
            res[f"sendrecv_{dt}"] = bool(torch.equal(o, base * ((rank - 1) % world + 1)))
        # the asynchronous forms through the Communicator (communicator stream + events)
        t = torch.full((1000,), float(rank), dtype=torch.float64, device=dev)
        comm.broadcast_async(t, world - 1).wait()
        res["bcast_async_last_root"] = bool((t == world - 1).all().item())
        comm.synchronize()
        res["unique_id_rank"] = rank
        res["ok"] = all(v for k, v in res.items() if isinstance(v, bool))
        C.destroy()
    except Exception:
        res["ok"] = False
        res["traceback"] = traceback.format_exc()
    (Path(outdir) / f"ops{rank}.json").write_text(json.dumps(res, indent=1))


def rbt_timed(rank, world, port, outdir, n, seed):
    """DistributedRBT over RCCL, graph-replayed: three solves (eager,
    captured, replayed); x of the last to x{rank}.pt, [graph, steps, berr,
    fallback, replay seconds] to meta{rank}.txt."""
    import time

    import torch

    from gelim.parallel import DistributedRBT
    from gelim.parallel import comm as C

    try:
        comm = _init(rank, world, port, "nccl")
        d = DistributedRBT(comm, n, single_fast_path=False)
        dt = None
        for _ in range(3):
            loc = d.generate_random(seed=seed)
            comm.synchronize()
            comm.barrier()
            t0 = time.perf_counter()
            x = d.solve_(loc)
            comm.synchronize()
            dt = time.perf_counter() - t0
        torch.save(x.cpu(), Path(outdir) / f"x{rank}.pt")
        (Path(outdir) / f"meta{rank}.txt").write_text(f"{d.graph} {d.last_steps} {d.last_berr} {d.last_fallback} {dt}")
        d.close()
        C.destroy()
    except Exception:
        (Path(outdir) / f"err{rank}.txt").write_text(traceback.format_exc())
        raise
