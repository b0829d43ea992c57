"""Distributed Gaussian elimination CLI — the MI355X counterpart of the
reference's MPI programs (OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c and
gauss_external_input.c), launched with torchrun, one rank per GPU over RCCL
(gloo + CPU ranks with --device cpu).

Internal mode (no FILE): the synthetic system A[i][j] = 2 min(i+1, j+1),
b[i] = i (gauss_internal_input.c:53-63), size -s N (default 2048); prints the
reference's `Application time: %f Secs` on rank 0, timer including the
initialisation like the reference (MPIi:322-334).

External mode (FILE = .dat or data/*.coo.npz): b = A (1..n)
(gauss_external_input.c:90-108); prints `Time:  %f seconds` (elimination +
back substitution, the reference times computeGauss only, MPIe:356-365) and
`Error: %e` (MPIe:371-378).

Unlike the reference's master/worker scheme (rank 0 ships full rows out and
back every pivot step), the matrix is resident and
column block-cyclic: one panel broadcast per block (parallel/dist_gauss.py).

--algo rbt runs the randomised block-LDU engine instead (parallel/dist_rbt.py:
random butterfly transform, no pivot chain, fp64 refinement, partial-
pivoting fallback), the distributed form of `--backend=hip-rbt`.

stdout is the MPI programs' own lines and nothing else: internal mode
`Application time: %f Secs` (plus `Max error vs exact solution` with
--verify), external mode `Time:  %f seconds` and `Error: %e`.

--emulate P runs P ranks as threads of this one process on one device (the
emulated communicator, parallel/emulated.py) — the distributed algorithm on a
single GPU.  --checkpoint-dir / --checkpoint-every / --resume save and resume
the elimination at panel boundaries (utils/checkpoint.py).
"""
from __future__ import annotations

import argparse
import sys
import time

import torch

from .. import _native
from ..ops.gauss import error_metric
from ..ops.init import augment_with_rhs
from ..parallel import comm as C
from ..parallel.dist_gauss import DistributedGauss
from ..utils import io
from ..utils.report import json_line


def parse(argv=None):
    p = argparse.ArgumentParser(prog="gelim.cli.dist_gauss", description=__doc__.split("\n\n")[0])
    p.add_argument("file", nargs="?", help=".dat or .coo.npz matrix (external mode)")
    p.add_argument("-s", "--size", type=int, default=2048, help="order of the synthetic system (internal mode)")
    p.add_argument("--block", type=int, default=None,
                   help="column block width D of the block-cyclic layout (default: 256 on GPUs, 64 on CPUs)")
    p.add_argument("-t", "--threads", type=int, default=None, metavar="N",
                   help="the reference's -t: here the number of ranks (GPUs) -- set by the launcher "
                        "(torchrun --nproc-per-node N); a mismatch is reported, not silently ignored")
    p.add_argument("--pivot", default="partial", choices=["partial", "zero"])
    p.add_argument("--algo", default="gauss", choices=["gauss", "rbt"],
                   help="gauss: partial pivoting (DistributedGauss); rbt: randomised block LDU (DistributedRBT)")
    p.add_argument("--device", default=None, help="cpu | cuda (default: cuda when visible)")
    p.add_argument("--warmup", type=int, default=0, help="untimed solves before the timed one")
    p.add_argument("--verify", action="store_true", help="print the max error against the exact solution")
    p.add_argument("--json", action="store_true", help="also print one JSON result line")
    p.add_argument("--emulate", type=int, default=0, metavar="P",
                   help="run P emulated ranks (threads) in this process on one device")
    p.add_argument("--checkpoint-dir", default=None, help="save panel-boundary checkpoints here")
    p.add_argument("--checkpoint-every", type=int, default=8, help="blocks between checkpoints")
    p.add_argument("--resume", action="store_true", help="resume from --checkpoint-dir")
    return p.parse_args(argv)


def load_global(path: str) -> torch.Tensor:
    if path.endswith(".npz"):
        n, r, c, v = io.load_coo_npz(path)
        return io.coo_to_dense(n, r, c, v)
    return io.read_dat(path)


def synthetic_local(dg: DistributedGauss) -> torch.Tensor:
    """Each rank builds only its own columns of the internal system."""
    L, n = dg.layout, dg.n
    loc = dg.empty_local()
    i = torch.arange(1, n + 1, dtype=torch.float64, device=dg.device).view(n, 1)
    for g in L.local_blocks(dg.comm.rank):
        c = L.local_col(g)
        w = max(0, min(L.width(g), n - g * L.D))  # real columns (GPU ranks pad to a multiple of 32)
        if w == 0:
            continue
        j = torch.arange(g * L.D + 1, g * L.D + w + 1, dtype=torch.float64, device=dg.device).view(1, w)
        loc[:n, c:c + w] = 2.0 * torch.minimum(i, j)
    loc[:n, dg.nloc] = torch.arange(n, dtype=torch.float64, device=dg.device)
    dg._pad_identity(loc)
    return loc


def synthetic_local_rbt(d) -> torch.Tensor:
    """The internal system in DistributedRBT's layout (local column jl is
    global column d.gcol[jl]; identity padding)."""
    n = d.n
    loc = d.empty_local()
    real = (d.gcol < n).nonzero().flatten()
    i = torch.arange(1, n + 1, dtype=torch.float64, device=d.device).view(n, 1)
    j = (d.gcol[real] + 1).to(torch.float64).view(1, -1)
    loc[:n, real] = 2.0 * torch.minimum(i, j)
    loc[:n, d.nloc] = torch.arange(n, dtype=torch.float64, device=d.device)
    d._pad_identity(loc)
    return loc


def make_solver(args, comm, n: int):
    """(solver, local-system builder for the internal mode, block width)."""
    if args.algo == "rbt":
        from ..parallel.dist_rbt import NB, DistributedRBT

        if args.checkpoint_dir:
            raise SystemExit("--checkpoint-dir is supported by --algo gauss only")
        d = DistributedRBT(comm, n)
        return d, (lambda: synthetic_local_rbt(d)), NB
    dg = DistributedGauss(comm, n, block=args.block, pivot=args.pivot)
    return dg, (lambda: synthetic_local(dg)), dg.layout.D


def main(argv=None) -> int:
    args = parse(argv)
    if args.emulate and args.emulate > 1:
        from ..parallel.emulated import run_emulated

        dev = args.device or ("cuda:0" if torch.cuda.is_available() else "cpu")
        return max(run_emulated(args.emulate, lambda comm: run(args, comm), device=dev))
    comm = C.init_from_env(device=args.device)
    ok = False
    try:
        rc = run(args, comm)
        ok = True
        return rc
    finally:
        # a failed rank (exception, CommFailure from the watchdog) aborts its
        # communicators instead of waiting for peers that may be gone
        C.destroy(abort=not ok)


def run(args, comm) -> int:
    dev = comm.device
    if args.threads is not None and args.threads != comm.world_size and comm.rank == 0:
        print(f"note: -t {args.threads} requests {args.threads} ranks but this job has {comm.world_size} "
              f"(launch with `torchrun --nproc-per-node {args.threads} -m gelim.cli.dist_gauss ...`, or "
              f"--emulate {args.threads} for threads on one device); running with {comm.world_size}",
              file=sys.stderr, flush=True)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        comm.barrier()

    rc = 0
    try:
        if args.file is None:
            n = args.size
            dg, build, D = make_solver(args, comm, n)
            for _ in range(args.warmup):
                dg.solve_(build())
            sync()
            ck = dg.checkpointer(args.checkpoint_dir, args.checkpoint_every) if args.checkpoint_dir else None
            t0 = time.perf_counter()
            loc = build()
            x = dg.solve_(loc, ckpt=ck, resume=args.resume) if ck else dg.solve_(loc)
            sync()
            dt = time.perf_counter() - t0
            if comm.rank == 0:
                print(f"Application time: {dt:f} Secs", flush=True)
                err = None
                if args.verify:
                    exact = torch.zeros(n, dtype=torch.float64)
                    exact[0], exact[-1] = -0.5, 0.5
                    err = float((x.cpu() - exact).abs().max())
                    print(f"Max error vs exact solution: {err:e}")
                if args.json:
                    json_line({"program": "dist_gauss_internal", "n": n, "ranks": comm.world_size,
                                     "algo": args.algo, "block": D, "time_s": dt, "max_abs_error": err,
                                     "backend": comm.backend, "device": dev.type})
        else:
            A = load_global(args.file)
            n = A.shape[0]
            aug = augment_with_rhs(A)
            dg, _, D = make_solver(args, comm, n)
            for _ in range(args.warmup):
                dg.solve_(dg.scatter_from_global(aug))
            loc = dg.scatter_from_global(aug)
            ck = dg.checkpointer(args.checkpoint_dir, args.checkpoint_every) if args.checkpoint_dir else None
            sync()
            t0 = time.perf_counter()
            x = dg.solve_(loc, ckpt=ck, resume=args.resume) if ck else dg.solve_(loc)
            sync()
            dt = time.perf_counter() - t0
            if comm.rank == 0:
                err = error_metric(x)
                # exactly the MPI program's two lines, no header (gauss_mpi/gauss_external_input.c:369,378)
                print(f"Time:  {dt:f} seconds")
                print(f"Error: {err:e}", flush=True)
                if args.json:
                    json_line({"program": "dist_gauss_external", "file": args.file, "n": n,
                                     "ranks": comm.world_size, "algo": args.algo, "block": D, "time_s": dt,
                                     "error": err, "backend": comm.backend, "device": dev.type})
    except _native.SingularMatrixError:
        if comm.rank == 0:
            print("The matrix is singular", file=sys.stderr)
        rc = 255  # the reference's exit(-1)
    return rc


if __name__ == "__main__":
    sys.exit(main())
