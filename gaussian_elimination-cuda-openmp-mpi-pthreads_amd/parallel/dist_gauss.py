"""Distributed Gaussian elimination across GPUs (one process per GPU, RCCL).

Replaces the reference's MPI master/worker program
(OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:124-255), where rank 0 owns
the whole matrix and ships full rows out and back every pivot step
(~8 n^3 bytes of traffic).  Here the data is resident and
owner-computes:

Layout: 1-D block-cyclic by COLUMNS, block width D.  Global column block g
lives on rank g % P as local block g // P.  The right-hand side b is
replicated on every rank as one extra local column, so every rank can apply
each panel's row operations to its own copy.

Factorisation, per global block g (k = g*D, owner o = g % P):
  1. owner factors its m x D panel locally (register-resident panel kernel,
     inner sub-panels + MFMA updates restricted to the panel);
  2. ONE broadcast from o of [panel ; pivots] (m+1 x D doubles) — the pivot
     search never leaves the owner because a column block is never split,
     so there is no per-column collective at all;
  3. every rank applies the panel to its trailing local columns (row swaps +
     TRSM + fp64 MFMA GEMM) and to its replica of b.
  => n/D broadcasts of O(n D) bytes instead of 2n small collectives.

Back substitution, per super-block of S = P*D columns (one block per rank),
last to first:
  all_reduce (sum) of the S partial dot products of the ranks' processed
  columns, then every rank solves the S x S diagonal triangle (gathered once
  up front with one all_gather) redundantly, so the solution x ends up
  replicated on every rank (the reference's "allgather of the solution").
  => n/S small all_reduces.

GPU ranks use the wide-panel engine (D = 256 by default, a multiple of the
32-column leaf; the system is padded to a multiple of 32 with an identity
block, which never wins a pivot search): the owner factors its panel with
the multi-workgroup leaves (csrc/hip/dist_panel.hip, one native call per
step), the broadcast carries [panel | leaf pair lists], and the schedule has
lookahead (on at every rank count) with TWO streams per rank:

  main  (owner of g+1): [wait panel g] [apply g -> block g+1] [factor g+1]
                        [bcast g+1 ......]
  side  (every rank):   [wait panel g] [apply g -> the next block this rank
                        will factor] (event) [apply g -> every other column]

so an owner's leaf chain runs beside its own trailing update (the side
stream's kernels use a capped grid, leaving CUs free for the leaves --
plan.hip's big-engine rule), the broadcast of g+1 travels under both, and
the panel buffers rotate over three slots (a slot is refilled only after the
side stream has finished the panel that used it).  The reference's workers
likewise all update rows at every step while the master overlaps its own
B update with the transfers (gauss_mpi/gauss_internal_input.c:141-175).

The last <= 2048 columns (GPU, lookahead) are not eliminated panel by
panel: their fully updated trailing system is all_gathered once and solved
redundantly on every rank by the single-GPU 2048 engine (GaussSolver: fused
register-resident steps + resident LU, one graph replay), then y_top = b_top
- U[:K, K:] x_tail is one local GEMV per rank + one all_reduce, and the top
K columns are back-substituted as above.  At 8192 that replaces 8 latency-
bound panel rounds by one 4 ms solve.

Runs on CPU tensors with gloo as well (the native CPU building blocks, the
original D = 64 sub-panel path), which is how the multi-rank path is tested
without GPUs.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import torch

from .. import _native
from ..ops import lu
from ..utils.checkpoint import Checkpointer, maybe_inject_fault
from ..utils.tensors import padded_ld, ptr, side_stream, stream_handle
from .comm import Communicator


def inner_width(m: int, device_type: str) -> int:
    """Sub-panel width the register-resident GPU panel kernel supports for m
    rows (CPU: same partition so CPU and GPU runs agree op for op)."""
    for w, rows in ((16, 2048), (8, 4096), (4, 8192), (2, 16384)):
        if m <= rows:
            return w
    raise ValueError(f"panel of {m} rows exceeds the register-resident panel kernel")


@dataclass(frozen=True)
class ColumnLayout:
    n: int
    P: int
    D: int

    @property
    def nblocks(self) -> int:
        return math.ceil(self.n / self.D)

    def owner(self, g: int) -> int:
        return g % self.P

    def width(self, g: int) -> int:
        return min(self.D, self.n - g * self.D)

    def local_blocks(self, r: int) -> list[int]:
        return list(range(r, self.nblocks, self.P))

    def nloc(self, r: int) -> int:
        return sum(self.width(g) for g in self.local_blocks(r))

    def local_col(self, g: int) -> int:
        return (g // self.P) * self.D

    def first_local_col_after(self, g: int, r: int) -> int:
        """Local column offset of rank r's first block with global index > g."""
        q = max(0, -(-(g + 1 - r) // self.P))  # ceil((g+1-r)/P)
        return min(q * self.D, self.nloc(r))


LEAF = 32  # leaf width of the wide-panel engine (csrc/hip/biglu.hip)
TAIL_ROWS = 2048  # GPU: the trailing system of at most this order goes to the single-GPU 2048 engine
NBUF = 3  # GPU panel buffers in rotation
COMPOSE_MAX_ROWS = 160 * 1024 // 4 - 1  # biglu.hip compose_max_rows(): one int per panel row in LDS


class DistributedGauss:
    """Column block-cyclic distributed solver of one n x n system.

    block: columns per block (GPU default 256, a multiple of 32; CPU 64).
    lookahead: GPU path -- factor the next panel on the main stream while the
    trailing update runs on a side stream, and finish with the 2048 engine
    (default on; off while checkpointing, whose snapshots need quiet block
    boundaries, and for lookahead=False: one stream, every block a panel).
    tail: order of the trailing system handed to the single-GPU engine
    (default TAIL_ROWS; 0 = none)."""

    def __init__(self, comm: Communicator, n: int, block: int | None = None, pivot: str = "partial",
                 lookahead: bool | None = None, tail: int | None = None):
        if lookahead is None:
            lookahead = True
        self.device = comm.device
        self.wide = self.device.type == "cuda"
        if block is None:
            block = 256 if self.wide else 64
        if block < 1:
            raise ValueError("block must be >= 1")
        if self.wide and block % LEAF:
            raise ValueError(f"GPU blocks are multiples of the {LEAF}-column leaf (got {block})")
        self.comm, self.n, self.pivot, self.lookahead = comm, n, pivot, lookahead
        self.tail_rows = TAIL_ROWS if tail is None else int(tail)
        # GPU: the system is padded to a multiple of the leaf width
        self.n_pad = -(-n // LEAF) * LEAF if self.wide else n
        self.layout = ColumnLayout(self.n_pad, comm.world_size, block)
        r = comm.rank
        self.nloc = self.layout.nloc(r)
        self.ld = padded_ld(self.nloc + 1)
        D = self.layout.D
        self._info = torch.zeros(4, dtype=torch.int32, device=self.device)
        if self.wide:
            lib = _native.lib()
            self._slot = int(lib.gelim_dist_pair_slot())
            nl = D // LEAF
            self._nnet = int(lib.gelim_dist_net_ints())
            # [leaf pair lists | composed movement | composed? flag], in doubles
            self._npd = -(-(nl * self._slot + self._nnet + 2) // 2)
            self._bufs = [torch.empty(self.n_pad * D + self._npd, dtype=torch.float64, device=self.device)
                          for _ in range(NBUF)]
            self._side = side_stream(self.device)  # probed: never on the default stream's queue
            self._cap = int(lib.gelim_dist_side_cap(self.n_pad))
            self._tail_solver = None
            self._pairs = torch.zeros(nl * self._slot, dtype=torch.int32, device=self.device)
            self._ipiv = torch.zeros(self.n_pad + 64, dtype=torch.int32, device=self.device)
            self._ws = torch.zeros(int(lib.gelim_gpu_leaf_workspace_bytes()) // 8, dtype=torch.float64,
                                   device=self.device)
        else:
            self._buf = torch.empty((n + 1) * D, dtype=torch.float64, device=self.device)
            self._piv = torch.zeros(D + 64, dtype=torch.int32, device=self.device)
        self._xt = None  # solution of the tail system (GPU lookahead path), set by factor_
        self.last_issue_s = 0.0  # host time to issue the last lookahead schedule

    # -- data placement -----------------------------------------------------
    def empty_local(self) -> torch.Tensor:
        return torch.zeros((self.n_pad, self.ld), dtype=torch.float64, device=self.device)

    def _pad_identity(self, loc: torch.Tensor) -> None:
        """Rows / columns n .. n_pad-1 of the padded system: identity."""
        L, n = self.layout, self.n
        for g in L.local_blocks(self.comm.rank):
            c, w = L.local_col(g), L.width(g)
            for j in range(max(g * L.D, n), g * L.D + w):
                loc[j, c + j - g * L.D] = 1.0

    def scatter_from_global(self, aug: torch.Tensor) -> torch.Tensor:
        """Local storage from a full augmented system present on every rank
        (tests / small problems)."""
        L, n = self.layout, self.n
        loc = self.empty_local()
        for g in L.local_blocks(self.comm.rank):
            c, w = L.local_col(g), L.width(g)
            wr = max(0, min(w, n - g * L.D))
            if wr:
                loc[:n, c:c + wr] = aug[:, g * L.D:g * L.D + wr].to(self.device)
        loc[:n, self.nloc] = aug[:, n].to(self.device)
        self._pad_identity(loc)
        return loc

    def generate_random(self, seed: int = 0) -> torch.Tensor:
        """Each rank generates ONLY its own columns of the random system
        (bit-identical to ops.init.random_system's A) and b = A (1..n) via one
        all_reduce of the per-rank partial products."""
        L, n = self.layout, self.n
        loc = self.empty_local()
        lib = _native.lib()
        idx = torch.empty(self.nloc, dtype=torch.float64, device=self.device)
        idx.zero_()
        for g in L.local_blocks(self.comm.rank):
            c, w = L.local_col(g), L.width(g)
            w = max(0, min(w, n - g * L.D))  # real (unpadded) columns of the block
            if w == 0:
                continue
            view = loc[:n, c:c + w]
            if self.device.type == "cuda":
                _native.check(lib.gelim_gpu_init_random_block(ptr(view), loc.stride(0), 0, n, g * L.D, w,
                                                              seed, stream_handle(self.device)), "init_random_block")
            else:
                tmp = torch.empty((n, w), dtype=torch.float64)
                lib.gelim_init_random_block_f64(ptr(tmp), w, 0, n, g * L.D, w, seed)
                view.copy_(tmp)
            idx[c:c + w] = torch.arange(g * L.D + 1, g * L.D + w + 1, dtype=torch.float64, device=self.device)
        b = loc[:, :self.nloc] @ idx if self.nloc else torch.zeros(self.n_pad, dtype=torch.float64,
                                                                   device=self.device)
        self.comm.all_reduce(b)
        loc[:, self.nloc] = b
        self._pad_identity(loc)
        return loc

    # -- factorisation -------------------------------------------------------
    def _subpanels(self, m: int, wg: int):
        w_in = inner_width(m, self.device.type)
        so = 0
        while so < wg:
            ws = min(w_in, wg - so)
            yield so, ws
            so += ws

    def _factor_owned_panel(self, panel: torch.Tensor, k: int) -> torch.Tensor:
        """Blocked factorisation of the owner's m x wg panel in place; returns
        the pivots of each sub-panel relative to that sub-panel's top row."""
        m, wg = panel.shape
        piv = torch.zeros(wg, dtype=torch.int32, device=self.device)
        for so, ws in self._subpanels(m, wg):
            lu.panel_factor(panel[so:, so:so + ws], piv[so:so + ws], self._info, row0=k + so, pivot=self.pivot)
            if so + ws < wg:
                lu.swap_trsm(panel[so:, so + ws:], panel[so:so + ws, so:so + ws], piv[so:so + ws])
                if m > so + ws:
                    lu.gemm_update(panel[so + ws:, so + ws:], panel[so + ws:, so:so + ws],
                                   panel[so:so + ws, so + ws:])
        return piv

    def checkpointer(self, directory, every: int = 1) -> Checkpointer:
        """Panel-boundary checkpoints of this solve (utils/checkpoint.py)."""
        L = self.layout
        return Checkpointer(directory, self.comm, {"n": self.n, "D": L.D, "pivot": self.pivot,
                                                   "ld": self.ld}, every)

    def factor_(self, loc: torch.Tensor, ckpt: Checkpointer | None = None, resume: bool = False,
                fault_at_block: int | None = None) -> None:
        """Forward elimination of the distributed augmented system in place.

        ckpt: save the state every ckpt.every blocks; resume: continue from
        its last complete generation (loc is overwritten with the saved slab).
        fault_at_block / GELIM_FAULT_AT_BLOCK: raise InjectedFault on entering
        that block (fault injection for the resume tests)."""
        if self.wide:
            return self._factor_wide(loc, ckpt, resume, fault_at_block)
        L, n, r = self.layout, self.n, self.comm.rank
        self._info.zero_()
        g0 = 0
        if ckpt is not None and resume:
            st = ckpt.load()
            if st is not None:
                loc.copy_(st.loc.to(loc.device))
                self._info.copy_(st.info.to(self._info.device))
                g0 = st.block
        for g in range(g0, L.nblocks):
            maybe_inject_fault(g, r, fault_at_block)
            if ckpt is not None and g > g0 and ckpt.due(g):
                ckpt.save(g, loc, self._info)
            k, wg, o = g * L.D, L.width(g), L.owner(g)
            m = n - k
            buf = self._buf[:(m + 1) * wg].view(m + 1, wg)
            if r == o:
                c = L.local_col(g)
                panel = loc[k:, c:c + wg]
                piv = self._factor_owned_panel(panel, k)
                buf[:m].copy_(panel)
                buf[m].copy_(piv.to(torch.float64))
            self.comm.broadcast(buf, src=o)
            c0 = L.first_local_col_after(g, r)
            C = loc[k:, c0:self.nloc + 1]  # trailing local columns + replicated b
            if C.shape[1] == 0:
                continue
            pivs = buf[m].to(torch.int32)
            for so, ws in self._subpanels(m, wg):
                lu.swap_trsm(C[so:], buf[so:so + ws, so:so + ws], pivs[so:so + ws])
                if m > so + ws:
                    lu.gemm_update(C[so + ws:], buf[so + ws:m, so:so + ws], C[so:so + ws])

    # -- GPU: wide-panel engine with lookahead -----------------------------------
    def _panel_factor(self, loc: torch.Tensor, g: int, buf: torch.Tensor, leaf: int, upd_end: int = 0,
                      wait_ev: torch.cuda.Event | None = None) -> int:
        """Owner: factor block g (up to date) in place and pack [panel |
        pair lists] into buf; returns the next leaf counter.  upd_end: the
        leaves also update local columns [end of block g, upd_end) -- the
        next block, once wait_ev has passed (one-rank lookahead)."""
        L, n = self.layout, self.n_pad
        k, wg, lc = g * L.D, L.width(g), L.local_col(g)
        m = n - k
        lib = _native.lib()
        _native.check(lib.gelim_dist_panel_factor(ptr(loc), loc.stride(0), n, k, lc, wg, lu._pivot_code(self.pivot),
                                                  ptr(self._ipiv), ptr(self._pairs), ptr(self._info), ptr(self._ws),
                                                  leaf, upd_end, wait_ev.cuda_event if wait_ev is not None else None,
                                                  stream_handle(self.device)), "dist_panel_factor")
        buf[:m * wg].view(m, wg).copy_(loc[k:, lc:lc + wg])
        nl = wg // LEAF
        tail = buf[m * wg:m * wg + self._npd].view(torch.int32)
        ns = nl * self._slot
        tail[:ns].copy_(self._pairs[:ns])
        # the panel's row movement composed ONCE here, shipped with the panel:
        # every rank's apply is then one gather/scatter, not a per-column
        # replay of the leaves' lists (~90 us a call)
        ok = _native.check(lib.gelim_dist_panel_compose(n, k, nl, ptr(self._pairs), ptr(tail[ns:]),
                                                        stream_handle(self.device)), "dist_panel_compose")
        tail[ns + self._nnet].fill_(ok)
        return leaf + nl

    def _bsize(self, g: int) -> int:
        L = self.layout
        return (self.n_pad - g * L.D) * L.width(g) + self._npd

    def _panel_apply(self, loc: torch.Tensor, g: int, buf: torch.Tensor, cb: int, ce: int,
                     stream: torch.cuda.Stream | None = None, cap: int = 0) -> None:
        """Panel g (from buf) applied to local columns [cb, ce), on `stream`
        (default: the current one), every launch on at most `cap` CUs."""
        if ce <= cb:
            return
        L, n = self.layout, self.n_pad
        k, wg = g * L.D, L.width(g)
        m = n - k
        tail = buf[m * wg:m * wg + self._npd].view(torch.int32)
        ns = (wg // LEAF) * self._slot
        # composed or not is a host-side function of (m, wg): the same test as
        # gelim_dist_panel_compose, so no device read is needed here
        net_ok = self._net_ok(m, wg // LEAF)
        sh = stream.cuda_stream if stream is not None else stream_handle(self.device)
        _native.check(_native.lib().gelim_dist_panel_apply(ptr(loc), loc.stride(0), n, k, cb, ce, ptr(buf), wg, wg,
                                                           ptr(tail), ptr(tail[ns:]), int(net_ok), cap, sh),
                      "dist_panel_apply")

    def _net_ok(self, m: int, nleaves: int) -> bool:
        net_max = (self._nnet - 2) // 2
        return m <= COMPOSE_MAX_ROWS and nleaves * 2 * LEAF <= net_max

    def _block_at_local_col(self, c: int) -> int:
        """Global block index of this rank's local block starting at local column c."""
        return self.comm.rank + (c // self.layout.D) * self.layout.P

    def _panel_blocks(self, use_tail: bool) -> int:
        """Blocks eliminated as broadcast panels; the rest is the tail system."""
        L = self.layout
        if not use_tail or self.tail_rows <= 0:
            return L.nblocks
        return max(0, -(-(self.n_pad - self.tail_rows) // L.D))

    def _factor_lookahead(self, loc: torch.Tensor, G: int, fault_at_block: int | None) -> None:
        """Panels 0..G-1 with the two-stream lookahead schedule (module
        docstring); every column of this rank -- the tail's included --
        receives every panel.  One rank: block g+1's update by panel g is
        fused into panel g's leaves (plan.hip's form), so the next panel
        factorisation starts the moment this one ends."""
        L, r, comm = self.layout, self.comm.rank, self.comm
        if G == 0:
            return
        fuse = comm.world_size == 1
        t_issue = time.perf_counter()
        end = self.nloc + 1  # local columns + b
        main = torch.cuda.current_stream(self.device)
        side = self._side
        side.wait_stream(main)  # loc / buffers as the caller left them
        B = self._bufs
        nb = len(B)
        ev_avail = [torch.cuda.Event() for _ in range(G)]
        ev_first = [torch.cuda.Event() for _ in range(G)]
        ev_rest = [torch.cuda.Event() for _ in range(G)]

        def fused_end(g: int) -> int:  # update range of panel g's leaves (one rank): through block g+1
            return L.local_col(g + 1) + L.width(g + 1) if fuse and g + 1 < L.nblocks else 0

        leaf = 0
        handles = {}
        o = L.owner(0)
        if r == o:
            leaf = self._panel_factor(loc, 0, B[0], leaf, fused_end(0))
        handles[0] = comm.broadcast_async(B[0][:self._bsize(0)], src=o)
        for g in range(G):
            maybe_inject_fault(g, r, fault_at_block)
            buf = B[g % nb]
            handles.pop(g).wait()  # main waits for panel g
            ev_avail[g].record(main)
            c0 = L.first_local_col_after(g, r)
            nxt = g + 1 < G
            o1 = L.owner(g + 1) if nxt else -1
            # side first (its events must exist before main waits on them):
            # panel g on the next block this rank factors after g+1, then on
            # everything else; block g+1 is main's
            cs = c0 + (L.width(g + 1) if (o1 == r or (fuse and g + 1 < L.nblocks)) else 0)
            wf = L.width(self._block_at_local_col(cs)) if cs < self.nloc else 0
            side.wait_event(ev_avail[g])
            with torch.cuda.stream(side):
                self._panel_apply(loc, g, buf, cs, cs + wf, side, self._cap)
                ev_first[g].record(side)
                self._panel_apply(loc, g, buf, cs + wf, end, side, self._cap)
                ev_rest[g].record(side)
            if o1 == r:
                if not fuse:
                    # block g+1: its last update (panel g) on main, then its
                    # factorisation; panel g-1 reached it first on the side
                    # stream (ev_first[g-1])
                    if g >= 1:
                        main.wait_event(ev_first[g - 1])
                    self._panel_apply(loc, g, buf, c0, c0 + L.width(g + 1))
                if g + 1 >= nb:
                    main.wait_event(ev_rest[g + 1 - nb])  # its buffer slot is free again
                # fused: panel g+1's leaves update block g+2 once panel g has
                # reached it on the side stream (ev_first[g])
                leaf = self._panel_factor(loc, g + 1, B[(g + 1) % nb], leaf, fused_end(g + 1),
                                          ev_first[g] if fuse else None)
            if nxt:
                if o1 != r and g + 1 >= nb:
                    main.wait_event(ev_rest[g + 1 - nb])
                handles[g + 1] = comm.broadcast_async(B[(g + 1) % nb][:self._bsize(g + 1)], src=o1)
        main.wait_event(ev_rest[G - 1])
        self.last_issue_s = time.perf_counter() - t_issue  # host time to issue the schedule

    def _tail_solve(self, loc: torch.Tensor, G: int) -> None:
        """The trailing system (rows and columns from K = G*D, every panel
        applied) gathered onto every rank and solved by the single-GPU engine;
        sets self._xt (tail solution) and self._ytop (b_top - U[:K, K:] x_t)."""
        L, P, r, comm = self.layout, self.comm.world_size, self.comm.rank, self.comm
        D, n = L.D, self.n_pad
        K = G * D
        mt = n - K
        nt = L.nblocks - G
        per = -(-nt // P)
        mine_b = [b for b in L.local_blocks(r) if b >= G]
        mine = torch.zeros((per, mt, D), dtype=torch.float64, device=self.device)
        for i, b in enumerate(mine_b):
            c, w = L.local_col(b), L.width(b)
            mine[i, :, :w] = loc[K:, c:c + w]
        gathered = torch.empty((P, per, mt, D), dtype=torch.float64, device=self.device)
        comm.all_gather(gathered.view(-1), mine.view(-1))
        aug = torch.empty((mt, padded_ld(mt + 1)), dtype=torch.float64, device=self.device)
        for t in range(nt):
            b = G + t
            q = b % P
            first_q = G + ((q - G) % P)
            w = L.width(b)
            aug[:, t * D:t * D + w] = gathered[q, (b - first_q) // P, :, :w]
        aug[:, mt] = loc[K:, self.nloc]
        if self._tail_solver is None or self._tail_solver.n != mt:
            from ..models.gauss_solver import GaussSolver

            # emulated ranks are threads of one process on one device: a graph
            # capture in one thread would collide with the others' launches on
            # the shared legacy stream, so they launch the tail engine eagerly
            self._tail_solver = GaussSolver(mt, backend="hip", pivot=self.pivot, device=self.device,
                                            use_graph=self.comm.backend != "emulated")
        xt = self._tail_solver.solve(aug)
        tinfo = self._tail_solver.info()  # raises on a hand-off error of the tail engine
        if tinfo:
            col = torch.full_like(self._info[:1], K + tinfo)
            self._info[:1] = torch.where(self._info[:1] == 0, col, self._info[:1])
        contrib = torch.zeros(K, dtype=torch.float64, device=self.device)
        if K:
            for b in mine_b:
                c, w = L.local_col(b), L.width(b)
                contrib += loc[:K, c:c + w] @ xt[(b - G) * D:(b - G) * D + w]
        comm.all_reduce(contrib)
        self._ytop = loc[:K, self.nloc] - contrib
        self._xt = xt

    def _factor_wide(self, loc: torch.Tensor, ckpt: Checkpointer | None, resume: bool,
                     fault_at_block: int | None) -> None:
        L, r, comm = self.layout, self.comm.rank, self.comm
        self._info.zero_()
        self._ws.zero_()
        self._xt = None
        if self.lookahead and ckpt is None:
            G = self._panel_blocks(use_tail=True)
            self._factor_lookahead(loc, G, fault_at_block)
            if G < L.nblocks:
                self._tail_solve(loc, G)
            return
        g0 = 0
        if ckpt is not None and resume:
            st = ckpt.load()
            if st is not None:
                loc.copy_(st.loc.to(loc.device))
                self._info.copy_(st.info.to(self._info.device))
                g0 = st.block
        # single stream, every block a broadcast panel (lookahead off, or
        # checkpointing: snapshots are taken at quiet block boundaries)
        end = self.nloc + 1  # local columns + b
        leaf = 0
        B = self._bufs
        if g0 < L.nblocks:
            maybe_inject_fault(g0, r, fault_at_block)
            o = L.owner(g0)
            if r == o:
                leaf = self._panel_factor(loc, g0, B[g0 & 1], leaf)
            h = comm.broadcast_async(B[g0 & 1][:self._bsize(g0)], src=o)
        for g in range(g0, L.nblocks):
            h.wait()
            buf = B[g & 1]
            self._panel_apply(loc, g, buf, L.first_local_col_after(g, r), end)
            if g + 1 < L.nblocks:
                maybe_inject_fault(g + 1, r, fault_at_block)
                if ckpt is not None and ckpt.due(g + 1):
                    ckpt.save(g + 1, loc, self._info)
                o1 = L.owner(g + 1)
                if r == o1:
                    leaf = self._panel_factor(loc, g + 1, B[(g + 1) & 1], leaf)
                h = comm.broadcast_async(B[(g + 1) & 1][:self._bsize(g + 1)], src=o1)

    def abort_code(self) -> int:
        """Hand-off error word of the GPU leaves (info[1], max over ranks):
        non-zero when a bounded spin timed out (code 5) or a row map left
        the system; every later leaf of that rank then returned early, so
        the factors are incomplete."""
        v = self._info[1:2].clone().to(torch.int64)
        self.comm.all_reduce(v, "max")
        return int(self.comm.item(v))

    def info(self) -> int:
        """First zero-pivot column + 1 over all ranks (0 = non-singular): each
        rank's own first one, combined with a min over the ranks that have
        one (0 maps to a sentinel past every column)."""
        v = self._info[:1].clone().to(torch.int64)
        sentinel = self.n_pad + 1
        v = torch.where(v == 0, torch.full_like(v, sentinel), v)
        self.comm.all_reduce(v, "min")
        val = int(self.comm.item(v))
        return 0 if val == sentinel else val

    # -- back substitution ----------------------------------------------------
    def backsolve(self, loc: torch.Tensor, y: torch.Tensor | None = None, ntop: int | None = None) -> torch.Tensor:
        """U x = y with U column-distributed, y replicated; returns x on every
        rank.  ntop: only the leading ntop x ntop triangle (a multiple of D;
        y then has ntop entries -- the tail path's y_top)."""
        L, P, D, r = self.layout, self.comm.world_size, self.layout.D, self.comm.rank
        n = L.n if ntop is None else ntop
        nblk = -(-n // D)
        if P == 1:  # local columns are the global ones: one back substitution
            yv = loc[:n, self.nloc] if y is None else y
            return lu.backsub(loc[:n, :n], yv)
        S = P * D
        nsuper = math.ceil(n / S)
        # one all_gather of every super-block's diagonal columns
        mine = torch.zeros((nsuper, S, D), dtype=torch.float64, device=self.device)
        for s in range(nsuper):
            g = s * P + r
            if g < nblk:
                s0, e = s * S, min((s + 1) * S, n)
                c, w = L.local_col(g), L.width(g)
                mine[s, :e - s0, :w] = loc[s0:e, c:c + w]
        gathered = torch.empty((P, nsuper, S, D), dtype=torch.float64, device=self.device)
        self.comm.all_gather(gathered.view(-1), mine.view(-1))
        y = (loc[:n, self.nloc] if y is None else y).contiguous()
        acc = torch.zeros((n, 1), dtype=torch.float64, device=self.device)  # -sum U x (own cols)
        x = torch.zeros(n, dtype=torch.float64, device=self.device)
        for s in reversed(range(nsuper)):
            s0, e = s * S, min((s + 1) * S, n)
            h = e - s0
            t = acc[s0:e, 0].clone()
            self.comm.all_reduce(t)
            rhs = y[s0:e] + t
            Uss = gathered[:, s, :h, :].permute(1, 0, 2).reshape(h, P * D)[:, :h].contiguous()
            xs = lu.backsub(Uss, rhs)
            x[s0:e] = xs
            g = s * P + r
            if g < nblk and s0 > 0:
                c, w = L.local_col(g), L.width(g)
                xp = xs[r * D:r * D + w].contiguous().view(w, 1)
                lu.gemm_update(acc[:s0], loc[:s0, c:c + w], xp)
        return x

    def solve_(self, loc: torch.Tensor, ckpt: Checkpointer | None = None, resume: bool = False,
               fault_at_block: int | None = None) -> torch.Tensor:
        """Factor + back-substitute (destroys loc); raises on a zero pivot."""
        self.factor_(loc, ckpt, resume, fault_at_block)
        code = self.abort_code()
        if code != 0:
            raise _native.GelimError(_native.E_HIP, f"GPU hand-off timed out or left the system (code {code}): "
                                                    "workgroups of a leaf were not co-resident; factors incomplete")
        if self.info() != 0:
            raise _native.SingularMatrixError(_native.E_SINGULAR, "The matrix is singular")
        if self._xt is not None:
            K = self.n_pad - self._xt.numel()
            xtop = self.backsolve(loc, self._ytop, K) if K else self._ytop
            return torch.cat([xtop, self._xt])[:self.n]
        return self.backsolve(loc)[:self.n]
