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

Runs on CPU tensors with gloo as well (the native CPU building blocks), which
is how the multi-rank path is tested without GPUs.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import _native
from ..ops import lu
from ..utils.checkpoint import Checkpointer, maybe_inject_fault
from ..utils.tensors import padded_ld, ptr, stream_handle
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


class DistributedGauss:
    """Column block-cyclic distributed solver of one n x n system."""

    def __init__(self, comm: Communicator, n: int, block: int = 64, pivot: str = "partial"):
        if block < 1:
            raise ValueError("block must be >= 1")
        self.comm, self.n, self.pivot = comm, n, pivot
        self.layout = ColumnLayout(n, comm.world_size, block)
        self.device = comm.device
        r = comm.rank
        self.nloc = self.layout.nloc(r)
        self.ld = padded_ld(self.nloc + 1)
        D = self.layout.D
        self._buf = torch.empty((n + 1) * D, dtype=torch.float64, device=self.device)
        self._piv = torch.zeros(D + 64, dtype=torch.int32, device=self.device)
        self._info = torch.zeros(4, dtype=torch.int32, device=self.device)

    # -- data placement -----------------------------------------------------
    def empty_local(self) -> torch.Tensor:
        return torch.zeros((self.n, self.ld), dtype=torch.float64, device=self.device)

    def scatter_from_global(self, aug: torch.Tensor) -> torch.Tensor:
        """Local storage from a full augmented system present on every rank
        (tests / small problems)."""
        L = self.layout
        loc = self.empty_local()
        for g in L.local_blocks(self.comm.rank):
            c, w = L.local_col(g), L.width(g)
            loc[:, c:c + w] = aug[:, g * L.D:g * L.D + w].to(self.device)
        loc[:, self.nloc] = aug[:, self.n].to(self.device)
        return loc

    def generate_random(self, seed: int = 0) -> torch.Tensor:
        """Each rank generates ONLY its own columns of the random system
        (bit-identical to ops.init.random_system's A) and b = A (1..n) via one
        all_reduce of the per-rank partial products."""
        L, n = self.layout, self.n
        loc = self.empty_local()
        lib = _native.lib()
        idx = torch.empty(self.nloc, dtype=torch.float64, device=self.device)
        for g in L.local_blocks(self.comm.rank):
            c, w = L.local_col(g), L.width(g)
            view = loc[:, c:c + w]
            if self.device.type == "cuda":
                _native.check(lib.gelim_gpu_init_random_block(ptr(view), loc.stride(0), 0, n, g * L.D, w,
                                                              seed, stream_handle(self.device)), "init_random_block")
            else:
                tmp = torch.empty((n, w), dtype=torch.float64)
                lib.gelim_init_random_block_f64(ptr(tmp), w, 0, n, g * L.D, w, seed)
                view.copy_(tmp)
            idx[c:c + w] = torch.arange(g * L.D + 1, g * L.D + w + 1, dtype=torch.float64, device=self.device)
        b = loc[:, :self.nloc] @ idx if self.nloc else torch.zeros(n, dtype=torch.float64, device=self.device)
        self.comm.all_reduce(b)
        loc[:, self.nloc] = b
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

    def info(self) -> int:
        """First zero-pivot column + 1 over all ranks (0 = non-singular)."""
        v = self._info[:1].clone().to(torch.int64)
        self.comm.all_reduce(v, "max")
        return int(v.item())

    # -- back substitution ----------------------------------------------------
    def backsolve(self, loc: torch.Tensor) -> torch.Tensor:
        """U x = y with U column-distributed, y replicated; returns x on every
        rank."""
        L, n, P, D, r = self.layout, self.n, self.comm.world_size, self.layout.D, self.comm.rank
        S = P * D
        nsuper = math.ceil(n / S)
        # one all_gather of every super-block's diagonal columns
        mine = torch.zeros((nsuper, S, D), dtype=torch.float64, device=self.device)
        for s in range(nsuper):
            g = s * P + r
            if g < L.nblocks:
                s0, e = s * S, min((s + 1) * S, n)
                c, w = L.local_col(g), L.width(g)
                mine[s, :e - s0, :w] = loc[s0:e, c:c + w]
        gathered = torch.empty((P, nsuper, S, D), dtype=torch.float64, device=self.device)
        self.comm.all_gather(gathered.view(-1), mine.view(-1))
        y = loc[:, self.nloc].contiguous()
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
            if g < L.nblocks and s0 > 0:
                c, w = L.local_col(g), L.width(g)
                xp = xs[r * D:r * D + w].contiguous().view(w, 1)
                lu.gemm_update(acc[:s0], loc[:s0, c:c + w], xp)
        return x

    def solve_(self, loc: torch.Tensor, ckpt: Checkpointer | None = None, resume: bool = False,
               fault_at_block: int | None = None) -> torch.Tensor:
        """Factor + back-substitute (destroys loc); raises on a zero pivot."""
        self.factor_(loc, ckpt, resume, fault_at_block)
        if self.info() != 0:
            raise _native.SingularMatrixError(_native.E_SINGULAR, "The matrix is singular")
        return self.backsolve(loc)
