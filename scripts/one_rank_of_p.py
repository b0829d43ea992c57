"""One rank of a P-rank DistributedRBT solve, replayed on ONE MI355X.

No multi-GPU node is reachable from this pool, so the distributed solver's
critical path at P = 8 cannot be timed directly.  This replays, on one GPU,
everything rank r of a P-rank run puts on its GPU PLUS every other rank's
chain work (the part of their work the critical path runs through):

  * rank r's own schedule, unchanged (parallel/dist_rbt.py
    _factor_lookahead): its 1/P share of the side-stream trailing updates,
    its own chain steps (every P-th block), its landing buffers;
  * for every block another rank owns, that owner's chain step on THIS GPU
    (DistributedRBT._foreign_chain / _foreign_side hooks): panel k applied to
    the block (its owner's "first" side GEMM, on a fourth stream), W, the
    diagonal-block update, the in-place 128 x 128 inverse and the column
    rest, on a rotating scratch slab;
  * every collective as a device-to-device copy of the same size on the
    communicator stream (ReplayComm): a broadcast received by rank r copies
    the virtual owner's scratch column into rank r's landing buffer after
    that owner's chain work (stream order), an all_reduce / all_gather moves
    its payload once / P times.

The GPU work of the factorisation is captured into a hipGraph and replayed,
as on the real run (host issue is not the bound).  What the replay does NOT
contain is xGMI transfer time: its copies run at HBM speed.  The report adds
it as a model -- per block, the small message's latency and, where the bulk
message is longer than the chain step, the difference -- for a range of link
latencies and bandwidths.  The chain work of the other ranks shares this GPU
with rank r's side updates, so the contention term is measured, not
modelled (and is pessimistic: on the real run each owner's chain competes
with its own 1/P side share only).

  python scripts/one_rank_of_p.py [--n 8192] [--P 8] [--rank 3] [--reps 5]

Values are not meaningful (the foreign columns are scratch); only time is.
Reference: OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:141-175 (the MPI
loop whose per-step traffic this schedule replaces)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.parallel.comm import Communicator, _Done  # noqa: E402
from gelim.parallel.dist_rbt import NB, DistributedRBT  # noqa: E402
from gelim.utils.tensors import dedicated_stream, ptr  # noqa: E402


class ReplayComm(Communicator):
    """Rank `rank` of a virtual world of `world` ranks on one GPU: every
    collective is a device copy of its payload (module docstring)."""

    capturable = True

    def __init__(self, world: int, rank: int, device: torch.device):
        super().__init__(rank=rank, world_size=world, device=device, backend="replay", group=None)
        self._scratch = None

    def _tmp(self, t: torch.Tensor) -> torch.Tensor:
        n = t.numel()
        if self._scratch is None or self._scratch.numel() < n * 8 or self._scratch.dtype != t.dtype:
            self._scratch = torch.empty(max(n, 1 << 20), dtype=t.dtype, device=self.device)
        return self._scratch[:n]

    def broadcast(self, t, src):
        if src != self.rank:
            t.view(-1).copy_(self._tmp(t))
        return t

    def broadcast_async(self, t, src):
        if src == self.rank:
            return _Done()
        return self._on_comm_stream(lambda s: t.view(-1).copy_(self._tmp(t)), t)

    def copy_async(self, dst: torch.Tensor, src: torch.Tensor):
        return self._on_comm_stream(lambda s: dst.copy_(src), dst, src)

    def all_reduce(self, t, op="sum"):
        self._tmp(t).copy_(t.view(-1))
        return t

    def all_gather(self, out, t):
        flat, n = out.view(-1), t.numel()
        for q in range(self.world_size):
            flat[q * n:(q + 1) * n].copy_(t.reshape(-1))
        return out

    def all_gather_async(self, out, t):
        self.all_gather(out, t)
        return _Done()

    def barrier(self):
        pass


class OneRankOfP(DistributedRBT):
    """DistributedRBT as rank r of P, with the other ranks' chain work
    replayed here (see the module docstring)."""

    def __init__(self, comm: ReplayComm, n: int, graph: bool = True, native_exec: bool = True):
        super().__init__(comm, n, single_fast_path=False, graph=graph, native_exec=native_exec)
        dev = self.device
        self._fs = [torch.randn(self.np, NB, dtype=torch.float64, device=dev) for _ in range(3)]
        self._Wf = torch.zeros((NB, NB), dtype=torch.float64, device=dev)
        self._Wfs = torch.zeros((2, NB, NB), dtype=torch.float64, device=dev)  # the native replay's W ring
        self._finfo = torch.zeros(1, dtype=torch.int32, device=dev)
        self._aux = dedicated_stream(dev, "aux")
        self._side_ev: dict[int, torch.cuda.Event] = {}
        self._ship_ev: dict[int, list] = {}

    def _patch_exec_args(self, a) -> None:
        """The native executor's replay mode (csrc/hip/drbt_exec.hip): the
        same foreign chain steps and copies as the hooks below."""
        a.replay = 1
        for i, f in enumerate(self._fs):
            a.F[i] = ptr(f)
        a.aux = self._aux.cuda_stream
        a.Wfs, a.finfo = ptr(self._Wfs), ptr(self._finfo)

    def _inv(self, blk: torch.Tensor, col: int) -> None:
        _native.check(_native.lib().gelim_rbt_block_inverse(ptr(blk), NB, col, ptr(blk), ptr(self._finfo),
                                                            self._sh()), "rbt_block_inverse")

    def _foreign_side(self, k, col, hs, hb):
        t = k + 2  # the block whose owner applies panel k to it first
        if t >= self.nb or t % self.P == self.rank:
            return
        f = self._fs[t % 3]
        aux = self._aux
        aux.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(aux):
            hs.wait()
            if hb is not None:
                hb.wait()
            for h in self._ship_ev.pop(t - 3, []):  # the scratch slab's previous column has been shipped
                h.wait()
            self._gemm_bm(self._Wfs[0], False, col[:NB], f[k * NB:(k + 1) * NB], False, NB, 1.0, False, aux)
            self._gemm_bm(f[(k + 1) * NB:], False, col[NB:], self._Wfs[0], False, NB, -1.0, True, aux)
            ev = torch.cuda.Event()
            ev.record(aux)
        self._side_ev[t] = ev

    def _foreign_chain(self, k, col, hb):
        t = k + 1
        f = self._fs[t % 3]
        if k < 0:
            self._inv(f[:NB], 0)
            return
        main = torch.cuda.current_stream(self.device)
        ev = self._side_ev.pop(t, None)
        if ev is not None:
            main.wait_event(ev)
        self._gemm_bm(self._Wf, False, col[:NB], f[k * NB:(k + 1) * NB], False, NB, 1.0, False)
        self._gemm_bm(f[t * NB:(t + 1) * NB], False, col[NB:2 * NB], self._Wf, False, NB, -1.0, True)
        self._inv(f[t * NB:(t + 1) * NB], t * NB)
        if (t + 1) * NB < self.np:
            if hb is not None:
                hb.wait()  # the rest of column k (as the owner's main stream waits for it)
            self._gemm_bm(f[(t + 1) * NB:], False, col[2 * NB:], self._Wf, False, NB, -1.0, True)

    def _ship(self, k):
        if k % self.P == self.rank:
            return super()._ship(k)
        dst = self._col(k).reshape(-1)
        src = self._fs[k % 3][k * NB:].reshape(-1)
        sm = self._small(k) * NB
        hs = self.comm.copy_async(dst[:sm], src[:sm])
        hb = self.comm.copy_async(dst[sm:], src[sm:dst.numel()]) if dst.numel() > sm else None
        self._ship_ev[k] = [h for h in (hs, hb) if h is not None]
        return hs, hb

    def factor_(self, loc):
        self._side_ev.clear()
        self._ship_ev.clear()
        return super().factor_(loc)


def time_it(fn, reps: int) -> list[float]:
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append(time.perf_counter() - t0)
    return out


def model(n: int, P: int, t_factor: float, t_apply: float, t_resid: float, corrections: int,
          lat_us: float, bw_gbs: float, t_chain_step: float) -> dict:
    """Measured replay + the xGMI terms the replay cannot contain."""
    npad = -(-n // (512 * P)) * (512 * P)
    nb = npad // NB
    link = 0.0
    for k in range(1, nb):
        small = min(2 * NB, npad - k * NB) * NB * 8
        rest = max(0, npad - k * NB - 3 * NB) * NB * 8
        t_small = lat_us * 1e-6 + small / (bw_gbs * 1e9)
        t_rest = lat_us * 1e-6 + rest / (bw_gbs * 1e9)
        # the chain waits for the small message [Dinv_k; L_{k+1,k}]; the
        # next-row message (one block, shipped beside the owner's inverse)
        # lands under the next owner's inverse; the column rest is first
        # needed two chain steps later (its first block feeds next_{k+1},
        # csrc/hip/drbt_exec.hip), so it costs only what it takes beyond that
        link += t_small + max(0.0, t_rest - 2 * t_chain_step)
    ns = npad // (NB * P)
    solve_lat = 2 * ns * (lat_us * 1e-6 + NB * P * 8 / (bw_gbs * 1e9))  # one all_reduce per super-block, 2 directions
    applies = 1 + corrections
    total = t_factor + link + applies * (t_apply + solve_lat) + applies * t_resid
    return {"lat_us": lat_us, "bw_GBs": bw_gbs, "link_factor_ms": link * 1e3, "solve_link_ms": solve_lat * 1e3,
            "total_ms": total * 1e3}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--corrections", type=int, default=2)
    ap.add_argument("--json", default=None)
    ap.add_argument("--factor-only", action="store_true",
                    help="(profiling) after the timed factorisations, one more factorisation and nothing else")
    ap.add_argument("--no-graph", action="store_true", help="Python schedule: issue eagerly (no hipGraph replay)")
    ap.add_argument("--python-schedule", action="store_true",
                    help="the Python lookahead loop (hipGraph-replayed unless --no-graph) instead of the native "
                         "executor")
    ap.add_argument("--side-cap", type=int, default=None,
                    help="CUs the side stream's trailing GEMMs may use (default: the solver's choice)")
    a = ap.parse_args()
    if not 0 <= a.rank < a.P:
        raise SystemExit(f"--rank {a.rank} is not a rank of P = {a.P}")
    dev = torch.device("cuda:0")
    comm = ReplayComm(a.P, a.rank, dev)
    d = OneRankOfP(comm, a.n, graph=not a.no_graph, native_exec=not a.python_schedule)
    if a.side_cap is not None:
        d.side_cap = a.side_cap
    loc = d.generate_random(seed=5)
    for _ in range(3):  # eager, captured, replayed
        d.factor_(loc)
    assert (not a.python_schedule or a.no_graph or (d.graph and d._graphs.get("factor") is not None)), \
        "the factorisation was not captured"
    tf = time_it(lambda: d.factor_(loc), a.reps)
    if a.factor_only:
        time.sleep(0.05)
        d.factor_(loc)
        torch.cuda.synchronize()
        print(json.dumps({"factor_ms": [round(t * 1e3, 3) for t in tf]}), flush=True)
        return
    d._gather_solve_blocks()
    rhs = torch.randn(d.np, dtype=torch.float64, device=dev)
    for _ in range(3):
        d.apply(rhs)
    ta = time_it(lambda: d.apply(rhs), a.reps)
    x = torch.randn(d.np, dtype=torch.float64, device=dev)
    tr = time_it(lambda: d._residual(loc, x), a.reps)
    # the chain step alone (owner's view): small GEMMs + inverse, from a
    # one-block micro-run on this GPU with nothing else queued
    tfm, tam, trm = min(tf), min(ta), min(tr)
    chain_step = tfm / d.nb
    res = {"n": a.n, "P": a.P, "rank": a.rank, "np": d.np, "blocks": d.nb, "graph": d.graph,
           "schedule": "native executor" if d.native_exec else "python", "issue_ms": (d.last_issue_s or 0) * 1e3,
           "factor_ms": [round(t * 1e3, 3) for t in tf], "apply_ms": [round(t * 1e3, 3) for t in ta],
           "residual_ms": [round(t * 1e3, 3) for t in tr], "factor_min_ms": tfm * 1e3, "apply_min_ms": tam * 1e3,
           "residual_min_ms": trm * 1e3, "factor_per_block_us": chain_step * 1e6,
           "measured_total_ms": (tfm + (1 + a.corrections) * (tam + trm)) * 1e3,
           "models": [model(a.n, a.P, tfm, tam, trm, a.corrections, lat, bw, chain_step)
                      for lat, bw in ((10, 100), (15, 100), (25, 50), (25, 100))]}
    line = json.dumps(res)
    print(line, flush=True)
    if a.json:
        Path(a.json).write_text(line + "\n")
    d.close()


if __name__ == "__main__":
    main()
