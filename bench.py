"""Headline benchmark: wall-clock seconds per 2048x2048 Gaussian-elimination
solve (fp64, partial pivoting, forward elimination + back substitution) on
MI355X, with the 2048^2 fp32 matmul reported alongside.

BASELINE.json metric: "wall-clock sec + speedup-vs-sequential, 2048x2048
Gauss-elim & matmul".  Reference numbers: Gauss 2048^2 OpenMP
best 0.509428 s; matmul 2048^2 CUDA V2 end-to-end 0.114906 s.

One step = one complete solve of a fresh random 2048^2 system on every GPU:
the pristine system is copied into the solver's working buffer (the
elimination is in place), eliminated with the blocked LU (register-resident
panel + fp64 MFMA trailing GEMM) and back-substituted.  N GPUs = N ranks
(torchrun), each solving its own system per step (weak scaling, "dp" over
independent systems); the step time is the MAX over ranks and `value` is
that wall time.  Data: synthetic random U[-1,1) matrices (b = A (1..n)),
generated on device; weights/checkpoints do not apply.

Sections after the headline (first-class fields of the same line, each timed
between device syncs + barriers, max over ranks):
  headline_fresh_systems the headline solve over a rotation of > 256 MB of
                        fresh systems (the headline itself re-solves one
                        34 MB system, resident in the 256 MB MALL)
  matmul_2048           2048^2 fp32, reference timer scope, warm + cold first call
  dist_gauss_8192(_s)   ONE 8192^2 system over ALL N ranks (strong scaling)
  dist_gauss_8192_rbt(_s) the same system over ALL N ranks on the randomised
                        block-LDU engine (no pivot chain; parallel/dist_rbt.py)
  dist_gauss_2048(_s)   the headline's 2048^2 system over ALL N ranks (strong)
  dist_gauss_32768(_s)  ONE 32768^2 system over ALL N ranks, partial pivoting
                        (strong; the trailing update dominates at this size)
  dist_rbt_16384(_s)    ONE 16384^2 system over ALL N ranks, randomised engine
  dist_matmul_16384(_s) 16384^2 fp32 over ALL N ranks (strong scaling)
  gauss_8192_1gpu(_s)   one 8192^2 system per GPU on the single-GPU solver
  hip_pivot_2048        the per-pivot algorithm (fp64, fp32)
  gauss_rbt             the randomised no-pivoting engine at 2048 / 8192 / 16384: hip-rbt
                        (butterfly transform + fp64 block-LDU on the matrix cores +
                        fp64 refinement to a componentwise backward error <= 4 eps);
                        fp64-class answers by a different algorithm than the
                        headline's partial pivoting, so reported beside it
  external_matrices     the reference's .dat matrices vs its best OpenMP times
  host_seq              sequential denominators: the Gauss loop timed in every
                        run on this host, the ~40 s i-j-k matmul stored unless
                        --measure-seq (the source field says which)

  python bench.py [--gpus N --steps K --warmup W] [--n 2048] [--headline-only]

Output: ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

BASELINE_GAUSS_S = 0.509428  # OpenMP best, 2048^2 (OpenMP_and_MPI/Report.pdf p.4)
BASELINE_MATMUL_S = 0.114906  # CUDA V2 end-to-end, 2048^2 (CUDA_and_OpenMP/Report.pdf p.2)
HOST_SEQ_FILE = ROOT / "profiles" / "host_seq_times.json"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--size", "--n", dest="n", type=int, default=2048,
                   help="matrix order of the headline system (--n is an alias)")
    p.add_argument("--backend", default="hip", choices=["hip", "hip-pivot"])
    p.add_argument("--graph", type=int, default=0, help="replay the solve from a hipGraph (1) or launch eagerly (0)")
    p.add_argument("--no-matmul", action="store_true")
    p.add_argument("--headline-only", action="store_true",
                   help="skip the distributed / 8192 / hip-pivot / external-matrix sections")
    p.add_argument("--budget", type=float, default=400.0,
                   help="seconds the sections after the headline may take before the line is printed without "
                        "the missing ones (a hung collective never costs the headline)")
    p.add_argument("--hang-exit-code", type=int, default=0,
                   help="exit status when the budget watchdog fires after a complete headline (the JSON line then "
                        "carries a 'watchdog' field and stderr says which sections hung); 0 keeps a scaling point "
                        "whose headline is complete, CI can ask for non-zero")
    p.add_argument("--measure-seq", action="store_true",
                   help="time the reference sequential loops on this host (slow)")
    return p.parse_args()


EXTERNAL_OPENMP_BEST_S = {  # BASELINE.md, OpenMP external, best over threads (OpenMP_and_MPI/Report.pdf p.6-7)
    "jpwh_991": 0.084672, "orsreg_1": 0.600996, "sherman5": 1.957547, "saylr4": 2.956282, "sherman3": 11.584218,
    "memplus": None,  # n = 17758: shipped in every matrices_dense/ but never timed by the reference
}


def _timed(comm, torch, dev, fn, reps: int = 1) -> float:
    """Wall time of `reps` calls of fn, bracketed by device sync + barrier on
    both sides, MAX over ranks."""
    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        comm.barrier()

    sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    t = torch.tensor([(time.perf_counter() - t0) / reps], dtype=torch.float64, device=dev)
    comm.all_reduce(t, "max")
    return t.item()


def _section(out: dict, key: str, fn) -> None:
    """Run one bench section; a failure is recorded, never fatal."""
    try:
        out[key] = fn()
    except Exception as e:  # noqa: BLE001
        out[key] = {"error": repr(e)[:300]}


def launch_ranks(n: int, argv: list[str]) -> int:
    """`python bench.py --gpus N` without a torchrun environment: act as a
    pure launcher (no torch / gelim import, no GPU call in this process) and
    run torchrun with N ranks as a CHILD process, relaying rank 0's JSON line
    on stdout (everything else goes to stderr).  Returns non-zero if any rank
    failed or no JSON line arrived.  The counterpart of the reference's
    `mpirun -np P` (OpenMP_and_MPI/README.txt:23,46), which refuses P < 2
    ranks (gauss_mpi/gauss_internal_input.c:289-297)."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # torchrun's own parser prefix-matches options even after the script
    # path ("--n" would be read as an abbreviation of "--nnodes")
    argv = ["--size" + a[3:] if a == "--n" or a.startswith("--n=") else a for a in argv]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]
    env = dict(os.environ, GELIM_BENCH_LAUNCHER="self (bench.py -> torchrun child)")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    assert proc.stdout is not None
    for raw in proc.stdout:  # streamed, so long runs keep showing progress
        if raw.startswith("{") and '"metric"' in raw:
            line = raw.strip()
            print(line, flush=True)
        else:
            print(raw, end="", file=sys.stderr, flush=True)
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: torchrun exited with {rc}", file=sys.stderr)
        return rc
    if line is None:
        print("bench.py: no JSON line from rank 0", file=sys.stderr)
        return 1
    return 0


def main() -> None:
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    import torch
    import torch.distributed as dist

    import gelim
    from gelim.parallel import comm as C

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    comm = C.init_from_env(timeout_s=300)
    dev = comm.device
    rank, N = comm.rank, comm.world_size
    joined = dist.get_world_size() if dist.is_initialized() else 1
    if joined != args.gpus:
        raise SystemExit(f"bench.py: {joined} ranks joined the process group, expected {args.gpus}")
    n = args.n
    on_gpu = dev.type == "cuda"
    backend = args.backend if on_gpu else "omp"  # CPU ranks (gloo): the OpenMP reference loop

    def dsync():
        if on_gpu:
            torch.cuda.synchronize(dev)

    # a watchdog prints whatever has been measured if a section hangs (a
    # stuck collective), so the headline line is never lost.  The line then
    # carries a "watchdog" field naming the unfinished sections and stderr
    # says so; the exit status is --hang-exit-code (default 0: the headline
    # measurement itself is complete, and a multi-GPU point of the scaling
    # curve is not voided by an optional section), while a failure of the
    # headline raises before this is armed.
    import threading

    result: dict = {}
    printed = threading.Event()

    def emit() -> None:
        if rank == 0 and not printed.is_set():
            printed.set()
            print(json.dumps(result), flush=True)

    def watchdog() -> None:
        done = [k for k in result if isinstance(result[k], dict) and k != "config"]
        result["watchdog"] = (f"sections after the headline did not finish within {args.budget:.0f} s "
                              f"(finished: {', '.join(done) or 'none'}); the headline above is complete")
        emit()
        sys.stdout.flush()
        print(f"bench.py: WATCHDOG: {result['watchdog']}", file=sys.stderr, flush=True)
        os._exit(args.hang_exit_code)

    # -- headline: one independent 2048^2 system per GPU ----------------------
    src = gelim.random_system(n, seed=1234 + rank, device=dev)
    if on_gpu:
        solver = gelim.GaussSolver(n, backend=backend, pivot="partial", device=dev, use_graph=bool(args.graph))
    else:
        solver = gelim.GaussSolver(n, backend=backend, pivot="partial")
    x = None
    for _ in range(args.warmup):
        x = solver.solve(src)
    dsync()
    comm.barrier()
    dsync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        x = solver.solve(src)
    dsync()
    comm.barrier()
    dsync()
    elapsed = time.perf_counter() - t0

    def reduce_max(v: "torch.Tensor") -> None:
        # the headline's two reductions go through torch.distributed itself
        # (ProcessGroupNCCL = RCCL), not libgelim's communicators, so the
        # headline never depends on the solvers' transport
        if dist.is_initialized() and joined > 1:
            dist.all_reduce(v, op=dist.ReduceOp.MAX)

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    reduce_max(t)
    step_s = t.item() / args.steps
    err = torch.tensor([gelim.ops.gauss.error_metric(x)], dtype=torch.float64, device=dev)
    reduce_max(err)
    info = solver.info()
    solver.close()
    del src, x

    result.update({
        "metric": f"wall-clock sec per {n}x{n} Gauss-elim solve (fp64, partial pivoting, "
                  "elimination + back-substitution) [BASELINE: wall-clock sec + speedup-vs-sequential, "
                  "2048x2048 Gauss-elim & matmul]",
        "value": step_s,
        "unit": "s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": False,
        "scaling": "weak",
        "vs_baseline": step_s / BASELINE_GAUSS_S,
        "speedup_vs_baseline": BASELINE_GAUSS_S / step_s,
        "dtype": "fp64 (Gauss, reference precision); fp32 (matmul)",
        "data": "synthetic random U[-1,1) systems generated on device, b = A(1..n); reference .dat matrices "
                "for external_matrices",
        "config": {"model": f"gauss_elim_{n}x{n}_partial_pivot_{backend}", "global_batch": N,
                   "seq_len": n, "parallelism": f"dp{N} (one independent system per GPU per step)"},
        "backend": comm.backend,
        "world_size": joined,
        "device": str(dev) if on_gpu else "cpu",
        "launcher": os.environ.get("GELIM_BENCH_LAUNCHER",
                                   "external torchrun" if "WORLD_SIZE" in os.environ else "single process"),
        "throughput_solves_per_s": N / step_s,
        "gflops_per_gpu": (2.0 / 3.0) * n ** 3 / step_s * 1e-9,
        "max_error": err.item(),
        "singular": info != 0,
        # build provenance: the digest of the sources libgelim.so was compiled from, and whether it is this tree's
        "libgelim_source_digest": gelim._native.build_digest(),
        "libgelim_built_from_tree": gelim._native.build_digest() == gelim._native.source_digest(),
    })
    timer = threading.Timer(args.budget, watchdog)
    timer.daemon = True
    timer.start()

    if not on_gpu:
        result["sections"] = "GPU-only sections skipped (CPU ranks)"
    if on_gpu:
        # the headline re-solves ONE 34 MB system, which stays resident in the
        # 256 MB MALL: the same solve over a rotation of fresh systems
        # (> 256 MB in total, generated outside the timed region)
        _section(result, "headline_fresh_systems", lambda: bench_fresh(comm, gelim, torch, n, backend, args.steps))
    if not args.no_matmul and on_gpu:
        _section(result, "matmul_2048", lambda: bench_matmul(gelim, torch, dev))
    if not args.headline_only and on_gpu:
        # strong scaling over ALL ranks: the BASELINE.json multi-GPU configs
        _section(result, "dist_gauss_8192", lambda: bench_dist_gauss(comm, gelim, torch, 8192))
        _section(result, "dist_gauss_8192_rbt", lambda: bench_dist_rbt(comm, gelim, torch, 8192))
        # the headline's 2048 system over ALL ranks (strong scaling, SURVEY §7.4-5: latency-bound,
        # reported as measured): every block a broadcast panel, and the default form (the whole
        # 2048 system is the tail: one all_gather + the single-GPU engine on every rank)
        _section(result, "dist_gauss_2048", lambda: {
            "panels": bench_dist_gauss(comm, gelim, torch, 2048, tail=0),
            "tail_engine": bench_dist_gauss(comm, gelim, torch, 2048)})
        _section(result, "dist_matmul_16384", lambda: bench_dist_matmul(comm, gelim, torch, 16384))
        # large-n strong scaling (one system over ALL ranks), where the trailing
        # update -- not the pivot chain -- dominates: the points of the curve
        # where more GPUs should visibly win (one timed solve each)
        _section(result, "dist_gauss_32768", lambda: bench_dist_gauss(comm, gelim, torch, 32768))
        _section(result, "dist_rbt_16384", lambda: bench_dist_rbt(comm, gelim, torch, 16384))
        # single-GPU large systems (each rank its own: weak)
        _section(result, "gauss_8192_1gpu", lambda: bench_single(comm, gelim, torch, 8192, seed=77 + rank))
        # past the round-2 cap of 32768 rows per leaf (8.6 GB per system)
        _section(result, "gauss_32768_1gpu", lambda: bench_single(comm, gelim, torch, 32768, seed=78 + rank, reps=1))
        _section(result, "hip_pivot_2048", lambda: bench_pivot(comm, gelim, torch, n))
        _section(result, "gauss_rbt", lambda: bench_rbt(comm, gelim, torch))
        _section(result, "external_matrices", lambda: bench_external(comm, gelim, torch))
    hf = result.get("headline_fresh_systems")
    if isinstance(hf, dict) and "time_s" in hf:
        result["headline_fresh_systems_s"] = hf["time_s"]
    for key, short in (("dist_gauss_8192", "dist_gauss_8192_s"), ("dist_gauss_8192_rbt", "dist_gauss_8192_rbt_s"),
                       ("dist_gauss_32768", "dist_gauss_32768_s"), ("dist_rbt_16384", "dist_rbt_16384_s"),
                       ("dist_matmul_16384", "dist_matmul_16384_s"),
                       ("gauss_8192_1gpu", "gauss_8192_1gpu_s"), ("gauss_32768_1gpu", "gauss_32768_1gpu_s")):
        v = result.get(key)
        if isinstance(v, dict) and "time_s" in v:
            result[short] = v["time_s"]
    rb = result.get("gauss_rbt")
    if isinstance(rb, dict):
        for nn in ("2048", "8192", "16384"):
            v = rb.get(nn, {}).get("hip-rbt")
            if isinstance(v, dict) and "time_s" in v:
                result[f"gauss_{nn}_rbt_s"] = v["time_s"]
    d2 = result.get("dist_gauss_2048")
    if isinstance(d2, dict) and "panels" in d2:
        result["dist_gauss_2048_s"] = d2["panels"]["time_s"]
        result["dist_gauss_2048_tail_engine_s"] = d2["tail_engine"]["time_s"]
    dm = result.get("dist_matmul_16384")
    if isinstance(dm, dict) and "summa" in dm:
        result["dist_matmul_16384_summa_s"] = dm["summa"]["time_s"]

    # -- speedup vs the reference's sequential loops --------------------------
    # The sequential Gauss loop (~0.6 s at 2048) is timed in EVERY run on this
    # host; the i-j-k matmul (~40 s) only with --measure-seq, else stored.
    seq = None
    if rank == 0:
        if args.measure_seq:
            seq = measure_host_seq(n)
            seq["source"] = "measured in this run on this host (Gauss and matmul)"
        else:
            stored = json.loads(HOST_SEQ_FILE.read_text()) if HOST_SEQ_FILE.exists() else {}
            seq = measure_host_seq(n, matmul=False)
            if "matmul_2048_s" in stored:
                seq["matmul_2048_s"] = stored["matmul_2048_s"]
            seq["source"] = (f"gauss_{n}_s measured in this run on this host; matmul_2048_s STORED: "
                             f"{HOST_SEQ_FILE.relative_to(ROOT)} (measured {stored.get('measured_at', '?')} on "
                             f"{stored.get('host', '?')}); --measure-seq re-measures it (~40 s)")
    if seq and rank == 0:
        result["host_seq"] = seq
        if "gauss_2048_s" in seq and n == 2048:
            result["speedup_vs_seq"] = seq["gauss_2048_s"] / step_s
        mm = result.get("matmul_2048")
        if isinstance(mm, dict) and "end_to_end_s" in mm and "matmul_2048_s" in seq:
            mm["speedup_vs_seq_end_to_end"] = seq["matmul_2048_s"] / mm["end_to_end_s"]
            mm["speedup_vs_seq_kernel"] = seq["matmul_2048_s"] / mm["kernel_s"]
    timer.cancel()
    emit()
    C.destroy()


def bench_fresh(comm, gelim, torch, n: int, backend: str, steps: int) -> dict:
    """The headline solve, each step on a DIFFERENT system from a rotation of
    ceil(320 MB / system) random systems generated before the timed region,
    so no step finds its input in the MALL (the 256 MB last-level cache)."""
    dev = comm.device
    per = n * (n + 1) * 8
    k = max(2, -(-320 * 2 ** 20 // per))
    pool = [gelim.random_system(n, seed=4000 + i + 100 * comm.rank, device=dev) for i in range(k)]
    solver = gelim.GaussSolver(n, backend=backend, pivot="partial", device=dev)
    for a in pool[:2]:
        solver.solve(a)
    holder = {}
    reps = max(steps, k)

    def run():
        for i in range(reps):
            holder["x"] = solver.solve(pool[i % k])

    dt = _timed(comm, torch, dev, run) / reps
    err = gelim.ops.gauss.error_metric(holder["x"])
    solver.close()
    del pool
    return {"time_s": dt, "systems": k, "pool_mb": k * per / 2 ** 20, "solves": reps, "max_error": err}


def bench_matmul(gelim, torch, dev) -> dict:
    """2048^2 fp32 matmul with the reference's timer scope (allocation, H2D,
    kernel, D2H, free).  cold = the very first call of the process (module
    load, first allocations); warm = median of 5 after 2 warmups."""
    A, B = gelim.ops.matmul.reference_inputs(2048)
    A, B = A.pin_memory(), B.pin_memory()
    Ch = torch.empty_like(A).pin_memory()
    model = gelim.MatMul("mfma", dev)
    cold = model.run_reference_style(A, B, Ch).end_to_end_s
    for _ in range(2):
        model.run_reference_style(A, B, Ch)
    runs = [model.run_reference_style(A, B, Ch) for _ in range(5)]
    e2e = sorted(r.end_to_end_s for r in runs)[len(runs) // 2]
    ker = sorted(r.kernel_s for r in runs)[len(runs) // 2]
    ref = A.double() @ B.double()
    rel = ((Ch.double() - ref).abs().max() / ref.abs().max()).item()
    for _ in range(2):
        model.run_pipelined(A, B, Ch)
    pruns = [model.run_pipelined(A, B, Ch) for _ in range(5)]
    pe2e = sorted(r.end_to_end_s for r in pruns)[len(pruns) // 2]
    prel = ((Ch.double() - ref).abs().max() / ref.abs().max()).item()
    best = min(e2e, pe2e)
    return {"n": 2048, "end_to_end_s": best, "end_to_end_serial_s": e2e, "end_to_end_pipelined_s": pe2e,
            "end_to_end_cold_first_call_s": cold, "kernel_s": ker, "kernel_tflops": 2 * 2048 ** 3 / ker * 1e-12,
            "vs_reference_cuda_v2": BASELINE_MATMUL_S / best,
            "vs_reference_cuda_v2_cold": BASELINE_MATMUL_S / cold, "max_rel_err": max(rel, prel)}


def bench_dist_gauss(comm, gelim, torch, n: int, tail: int | None = None) -> dict:
    """The n^2 system distributed over ALL ranks (strong scaling; column
    block-cyclic, wide-panel leaves, RCCL broadcast with lookahead); second
    solve timed.  tail=0: every block is a broadcast panel (no trailing
    system handed to the single-GPU engine)."""
    from gelim.parallel import DistributedGauss

    dev = comm.device
    dg = DistributedGauss(comm, n, tail=tail)
    holder = {}

    def run():
        holder["x"] = dg.solve_(holder.pop("loc"))

    for _ in range(2):
        holder["loc"] = dg.generate_random(seed=99)
        dt = _timed(comm, torch, dev, run)
    x = holder["x"]
    return {"time_s": dt, "error": gelim.ops.gauss.error_metric(x), "ranks": comm.world_size,
            "tflops_total": (2.0 / 3.0) * n ** 3 / dt * 1e-12, "block": dg.layout.D,
            "lookahead": dg.lookahead, "layout": "1-D column block-cyclic",
            "broadcast_panels": dg._panel_blocks(use_tail=True), "tail_rows": dg.tail_rows}


def bench_dist_rbt(comm, gelim, torch, n: int) -> dict:
    """The n^2 system over ALL ranks with the randomised block-LDU engine
    (parallel/dist_rbt.py: butterfly transform local to each rank, one
    [Dinv_k | L_k] broadcast per 128-column block with lookahead, super-block
    solves, fp64 refinement on the original system; the factorisation loop
    and the applies replayed from hipGraphs with libgelim's RCCL
    communicators inside); third solve timed.  One
    rank: the single-GPU native solve of the same padded system, and the
    distributed schedule on that one rank beside it."""
    from gelim.parallel import DistributedRBT

    dev = comm.device

    def timed(d):
        holder = {}

        def run():
            holder["x"] = d.solve_(holder.pop("loc"))

        for _ in range(3):  # eager, captured into a hipGraph, replayed: the last is timed
            holder["loc"] = d.generate_random(seed=99)
            dt = _timed(comm, torch, dev, run)
        return dt, holder["x"]

    d = DistributedRBT(comm, n)
    dt, x = timed(d)
    out = {"time_s": dt, "error": gelim.ops.gauss.error_metric(x), "ranks": comm.world_size,
           "padded_order": d.np, "corrections": d.last_steps, "backward_error": d.last_berr,
           "fallback": d.last_fallback, "tflops_total": (2.0 / 3.0) * n ** 3 / dt * 1e-12,
           "path": "single-GPU native solve" if d.fast else "distributed schedule",
           "graph": bool(getattr(d, "graph", False)), "native_rccl": comm.native}
    d.close()
    if comm.world_size == 1:
        d1 = DistributedRBT(comm, n, single_fast_path=False)
        out["schedule_one_rank_s"], _ = timed(d1)
        d1.close()
    return out


def bench_dist_matmul(comm, gelim, torch, n: int) -> dict:
    """16384^2 fp32 matmul over ALL ranks (strong scaling), three
    decompositions timed side by side:
      allgather  A/C row blocks, B gathered in column chunks
                 (all_gather_into_tensor) under the MFMA GEMM, the own k-block
                 under the first gather (the default, `time_s`);
      summa      2-D pr x pc block decomposition (BASELINE.json config 5):
                 row / column sub-communicator broadcasts of A and B k-panels,
                 double-buffered and asynchronous under the GEMM of the
                 previous panel;
      ring       B blocks passed around a ring of batched isend/irecv
                 (more than one rank)."""
    from gelim.parallel import allgather_matmul, ring_matmul
    from gelim.parallel.dist_matmul import default_chunks, grid_shape, make_summa_groups, summa_matmul

    dev, P, r = comm.device, comm.world_size, comm.rank
    g = torch.Generator(device=dev).manual_seed(1 + r)
    Aloc = torch.randn(n // P, n, generator=g, device=dev)
    Bloc = torch.randn(n // P, n, generator=g, device=dev)
    out = {}
    for name, fn in (("allgather", allgather_matmul), ("ring", ring_matmul)):
        if name == "ring" and P == 1:
            continue
        fn(comm, Aloc, Bloc)
        dt = _timed(comm, torch, dev, lambda: fn(comm, Aloc, Bloc), reps=2)
        out[name] = {"time_s": dt, "tflops_total": 2 * n ** 3 / dt * 1e-12}
    out["allgather"]["chunks"] = default_chunks(P)
    del Aloc, Bloc
    pr, pc = grid_shape(P)
    Ablk = torch.randn(n // pr, n // pc, generator=g, device=dev)
    Bblk = torch.randn(n // pr, n // pc, generator=g, device=dev)
    groups = make_summa_groups(comm, pr, pc)
    summa_matmul(comm, Ablk, Bblk, (pr, pc), groups=groups)
    dt = _timed(comm, torch, dev, lambda: summa_matmul(comm, Ablk, Bblk, (pr, pc), groups=groups), reps=2)
    out["summa"] = {"time_s": dt, "tflops_total": 2 * n ** 3 / dt * 1e-12, "grid": f"{pr}x{pc}"}
    out["time_s"] = out["allgather"]["time_s"]
    out["algo"] = "allgather (chunked all_gather_into_tensor of B overlapped with the MFMA GEMM)"
    out["ranks"] = P
    return out


def bench_single(comm, gelim, torch, n: int, seed: int, reps: int = 3) -> dict:
    """One n^2 system per GPU on the single-GPU solver (n > 2048: wide-panel
    leaves + fp64 MFMA GEMM + the 2048 engine on the tail)."""
    dev = comm.device
    aug = gelim.random_system(n, seed=seed, device=dev)
    s = gelim.GaussSolver(n, backend="hip", device=dev)
    holder = {}
    s.solve(aug)
    dt = _timed(comm, torch, dev, lambda: holder.__setitem__("x", s.solve(aug)), reps=reps)
    res = {"time_s": dt, "tflops": (2.0 / 3.0) * n ** 3 / dt * 1e-12,
           "error": gelim.ops.gauss.error_metric(holder["x"]), "singular": s.info() != 0}
    s.close()
    return res


def bench_rbt(comm, gelim, torch) -> dict:
    """The randomised no-pivoting engine hip-rbt (each rank its own system):
    the whole solve (transform, factorisation, refinement) per call, with the
    refinement's correction count, its final componentwise backward error and
    whether it fell back to partial pivoting."""
    dev = comm.device
    out = {}
    for n in (2048, 8192, 16384):
        aug = gelim.random_system(n, seed=31 + n, device=dev)
        s = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
        holder = {}
        s.solve(aug)
        dt = _timed(comm, torch, dev, lambda: holder.__setitem__("x", s.solve(aug)), reps=3)
        out[str(n)] = {"hip-rbt": {"time_s": dt, "error": gelim.ops.gauss.error_metric(holder["x"]),
                                   "corrections": s.last_steps, "backward_error": s.last_berr,
                                   "fallback": s.last_fallback}}
        s.close()
        del aug
    return out


def bench_pivot(comm, gelim, torch, n: int) -> dict:
    """The reference's per-pivot algorithm on the GPU (hip-pivot: one pivot
    search + one elimination launch per column, graph-replayed), fp64 and
    fp32, zero-pivot (internal programs) and partial pivoting."""
    dev = comm.device
    aug = gelim.random_system(n, seed=5, device=dev)
    out = {}
    for dtype, tag in ((torch.float64, "fp64"), (torch.float32, "fp32")):
        s = gelim.GaussSolver(n, backend="hip-pivot", pivot="partial", dtype=dtype, device=dev)
        a = aug.to(dtype)
        holder = {}
        s.solve(a)
        dt = _timed(comm, torch, dev, lambda: holder.__setitem__("x", s.solve(a)), reps=3)
        out[tag] = {"time_s": dt, "error": gelim.ops.gauss.error_metric(holder["x"])}
        s.close()
    return out


def bench_external(comm, gelim, torch) -> dict:
    """GPU solve time of the reference's external .dat matrices (the
    Matrix-Market inputs of gauss_external_input, shipped as data/*.coo.npz)
    next to the reference's best OpenMP time.  The timed solve includes the
    copy-in of the system (like the headline)."""
    dev = comm.device
    out = {}
    if comm.rank == 0:
        for name, ref_s in EXTERNAL_OPENMP_BEST_S.items():
            A = gelim.utils.io.load_fixture(name)
            n = A.shape[0]
            aug = gelim.augment_with_rhs(A).to(dev)
            s = gelim.GaussSolver(n, backend="hip", device=dev)
            x = s.solve(aug, check=True)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(3):
                x = s.solve(aug)
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / 3
            out[name] = {"n": n, "time_s": dt, "error": gelim.ops.gauss.error_metric(x),
                         "reference_openmp_best_s": ref_s,
                         "speedup_vs_reference_openmp": ref_s / dt if ref_s else None}
            s.close()
            del aug, A
    comm.barrier()
    return out


def measure_host_seq(n: int, matmul: bool = True) -> dict:
    """The reference's sequential loops on this host (the speedup denominator,
    SURVEY.md §6 caveat): the external programs' partial-pivoting elimination
    (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182 run on one
    thread) and the i-j-k matmul (CUDA_and_OpenMP/Version-2/cuda_matmul.cu:28-39)."""
    import gelim

    aug = gelim.random_system(n, seed=1234)
    A = aug[:, :n].contiguous().clone()
    b = aug[:, n].contiguous().clone()
    t0 = time.perf_counter()
    gelim.ops.gauss.cpu_gauss_(A, b, "seq", "partial")
    gauss_s = time.perf_counter() - t0
    res = {f"gauss_{n}_s": gauss_s, "host": os.uname().nodename, "cpus": os.cpu_count(),
           "measured_at": time.strftime("%Y-%m-%dT%H:%M:%S")}
    if matmul:
        Am, Bm = gelim.ops.matmul.reference_inputs(2048)
        t0 = time.perf_counter()
        gelim.ops.cpu_matmul(Am, Bm)
        res["matmul_2048_s"] = time.perf_counter() - t0
    return res


if __name__ == "__main__":
    main()
