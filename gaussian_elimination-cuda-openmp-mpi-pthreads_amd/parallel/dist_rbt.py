"""Distributed randomised solver: the `hip-rbt` engine (random butterfly
transform + block LDU WITHOUT pivoting + fp64 refinement, csrc/hip/lu_mixed.hip)
over one process per GPU (RCCL).

Why a second distributed solver: the partial-pivoting DistributedGauss has
the owner of each block factor its panel alone, one global arg-max per
column, while the other ranks wait -- its critical path barely shrinks with
P (profiles/dist_gauss_8rank_critical_path.md).  Without pivoting there is no
per-column reduction at all: a block step is one 128 x 128 Gauss-Jordan
inverse plus GEMMs that every rank runs on its own columns, which is the
reference MPI program's "every worker updates rows at every step"
(OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-199) with resident data
and one broadcast per 128-column block instead of 2 (n - i) rows shipped per
pivot.

Layout: 128-column blocks, block g on rank g % P (a rank's blocks left to
right), the right-hand side replicated as one extra local column.  The order
is padded with an identity block to np, a multiple of 512 P: then every
butterfly column group {j, j + np/4, j + np/2, j + 3np/4} lies on one rank
and the transform M = U^T A V is local (csrc/hip/dist_rbt.hip).

Storage: column-block-major -- local block lb is its own contiguous np x 128
slab Mb[lb], so the column of block k from its diagonal block down is ONE
contiguous buffer and goes out in an in-place broadcast (no pack copy).  The
owner inverts the diagonal block IN PLACE: the slab's diagonal block holds
Dinv_k afterwards (the block-LDU factor never needs A_kk again), so the column
message is [Dinv_k; L_{k+1,k}; L_{k+2,k}; ...].

Factorisation (block k, owner o = k % P), two messages per block:
  small_k = [Dinv_k; L_{k+1,k}]   (256 x 128: all the next owner needs to
                                   update and invert its diagonal block)
  bulk_k  = L_{k+2.., k}          (the rest of the column, off the chain)
  owner of k+1 (main stream): wait small_k; W = Dinv_k M[k, k+1];
      M[k+1, k+1] -= L_{k+1,k} W; Dinv_{k+1} = M[k+1,k+1]^-1 in place (the
      chain: it needs nothing of bulk_k); then wait bulk_k;
      M[k+2.., k+1] -= L_{k+2..,k} W; broadcast small_{k+1}, bulk_{k+1}
  every rank (side stream): wait small_k + bulk_k; W = Dinv_k M[k, own
      cols]; M[>k, own cols] -= L_k W (its next block first, so the chain of
      the next step never waits for the rest)
The off-diagonal blocks stay in place as the block-LDU factor, the inverses
on their diagonal blocks.  Three landing buffers rotate on the receivers.
Critical path per block: small-message latency + two 128^3 GEMMs + the
inverse (+ the column rest when the bulk is late)
(profiles/dist_rbt_8rank_critical_path.md).

Solves (every apply of (LU)^-1, replicated vectors): super-blocks of P
blocks -- one block per rank, the same local block index s on every rank.
The super-diagonal S x S blocks (S = 128 P) and all inverses are all_gathered
once after the factorisation; then per super-block, one all_reduce of the S
partial sums, a redundant S x S block-triangular solve on every rank
(gelim_drbt_super_solve) and a local GEMV of the rank's own block column.
That is np / S collectives of S doubles per direction.

Refinement: x += (LU)^-1 (b - A x) on the ORIGINAL (padded) system until the
componentwise backward error max_i |r_i| / (|b| + |A||x|)_i <= 4 eps64 (one
all_reduce of [A_loc x_loc, |A_loc||x_loc|] per step), exactly the single-GPU
rule (gelim_mixed_solve); a non-finite inverse or a stall hands the system to
DistributedGauss (partial pivoting) with the same 128-column block layout.

One rank: the single-GPU native solve (gelim_mixed_solve) on the local
storage, which IS the padded augmented system (single_fast_path=False runs
the distributed schedule on one rank, for tests).

CPU ranks (gloo tests without a GPU) run the same schedule with torch CPU
ops standing in for the HIP kernels (dense butterflies, torch.linalg.inv,
matmul) -- the orchestration, layouts and collectives are identical.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .. import _native
from ..utils.tensors import ptr, side_stream, stream_handle
from .comm import Communicator

NB = 128  # block width (= the single-GPU engine's)
NBUF = 3  # broadcast buffers in rotation
SEED = 0x5EED  # butterfly seed (the single-GPU GaussSolver's)


def padded_order(n: int, P: int) -> int:
    """np: n rounded up to a multiple of 512 P (butterfly column groups local)."""
    q = 4 * NB * P
    return -(-n // q) * q


def butterfly_diagonals(npad: int, seed: int = SEED) -> tuple[np.ndarray, np.ndarray]:
    """U's and V's butterfly diagonals, 8 x npad/4 each: exp(r / 10), r uniform
    in [-1/2, 1/2] -- GaussSolver._init_mixed's draw for the same npad."""
    rng = np.random.default_rng(seed)
    ud = np.exp((rng.random(2 * npad) - 0.5) / 10.0)
    vd = np.exp((rng.random(2 * npad) - 0.5) / 10.0)
    return ud, vd


def butterfly_dense(d: np.ndarray, npad: int) -> torch.Tensor:
    """Dense npad x npad butterfly W with W[i + c h, i + q h] = W_i[c][q]
    (csrc/hip/rbt.h group_w), so U^T A V = W_u^T A W_v (CPU path, tests)."""
    h = npad // 4
    i = np.arange(h)
    r0, r0h, s0, s0h, ra, sa, rb, sb = (d[k * h:(k + 1) * h] for k in range(8))
    z = np.zeros(h)
    L0 = np.array([[r0, z, s0, z], [z, r0h, z, s0h], [r0, z, -s0, z], [z, r0h, z, -s0h]])  # 4 x 4 x h
    L1 = np.array([[ra, sa, z, z], [ra, -sa, z, z], [z, z, rb, sb], [z, z, rb, -sb]])
    Wg = 0.5 * np.einsum("ach,cbh->abh", L1, L0)  # W_i[a][b]
    W = np.zeros((npad, npad))
    for a in range(4):
        for b in range(4):
            W[i + a * h, i + b * h] = Wg[a, b]
    return torch.from_numpy(W)


import ctypes as _C


class _ExecArgs(_C.Structure):
    """gelim_drbt_args of csrc/hip/drbt_exec.hip (keep in sync)."""
    _fields_ = [("np", _C.c_int64), ("nloc", _C.c_int64), ("P", _C.c_int32), ("rank", _C.c_int32),
                ("Mb", _C.c_void_p), ("mbs", _C.c_int64), ("X", _C.c_void_p * 3), ("Wm", _C.c_void_p),
                ("Ws", _C.c_void_p), ("info", _C.c_void_p), ("main", _C.c_void_p), ("side", _C.c_void_p),
                ("comm", _C.c_void_p), ("rccl_small", _C.c_void_p), ("rccl_bulk", _C.c_void_p),
                ("side_cap", _C.c_int32), ("replay", _C.c_int32), ("F", _C.c_void_p * 3), ("aux", _C.c_void_p),
                ("Wfs", _C.c_void_p), ("finfo", _C.c_void_p)]


class DistributedRBT:
    """Randomised block-LDU solve of one n x n system over all ranks of comm."""

    def __init__(self, comm: Communicator, n: int, seed: int = SEED, lookahead: bool = True,
                 single_fast_path: bool = True, max_steps: int = 6, graph: bool = True, native_exec: bool = True):
        self.comm, self.n = comm, n
        self.P, self.rank = comm.world_size, comm.rank
        self.device = comm.device
        self.gpu = self.device.type == "cuda"
        self.lookahead = lookahead
        self.max_steps = max_steps
        self.np = padded_order(n, self.P)
        self.pad_ratio = self.np / max(1, n)
        if self.P > 1 and self.pad_ratio > 1.25:
            import warnings

            warnings.warn(f"DistributedRBT: n = {n} on {self.P} ranks is padded to {self.np} (a multiple of "
                          f"{4 * NB * self.P}): {self.pad_ratio ** 3:.1f}x the factorisation flops of n; "
                          "DistributedGauss or fewer ranks may be faster", RuntimeWarning, stacklevel=2)
        self.nb = self.np // NB
        self.nloc = self.np // self.P
        self.nbl = self.nb // self.P  # local blocks = super-blocks
        self.ld = self.nloc + 2       # b in column nloc; even, 16-byte rows
        self.fast = single_fast_path and self.P == 1 and self.gpu
        # hipGraph replay of the fixed schedules (factorisation loop, apply):
        # the host issue of one block -- ~15 launches, two collectives, their
        # events -- costs 120 us eagerly and 255 us with RCCL's host side,
        # more than the GPU chain of a block at 8 ranks
        # (profiles/dist_issue_r5.md).  Only where every op is a stream op:
        # libgelim's native RCCL or no collective at all (gloo and the
        # emulated ranks meet on the host; torch's ProcessGroupNCCL watchdog
        # aborts on collectives recorded during a capture).
        self.graph = graph and self.gpu and lookahead and (comm.backend == "none" or comm.native
                                                           or getattr(comm, "capturable", False))
        self._graphs: dict[str, torch.cuda.CUDAGraph | None] = {}
        # the lookahead factorisation issued natively (csrc/hip/drbt_exec.hip)
        # wherever every collective is libgelim's own RCCL (or there is none):
        # ~30 us of host time per block on the probed streams, instead of a
        # Python loop or a hipGraph whose replay remaps the streams' queues
        self.native_exec = (native_exec and self.gpu and lookahead
                            and (comm.backend == "none" or comm.native or getattr(comm, "capturable", False)))
        self._exec = None
        # CUs the bulk GEMMs beside the chain (side stream; the native
        # executor's rows below the chain, on the communicator stream) may
        # take, 0: all.  Uncapped they fill every CU's LDS (dgemm 64-tiles: 4
        # x 40 KB) and the chain's next kernel -- the inverse, a W product --
        # waits for the whole grid to be dispatched: 40-120 us per block in the
        # one-rank-of-8 replay (profiles/dist_rbt_replay_r6.md).  Capped, the
        # persistent form leaves 16 CUs free.  Only from 8 ranks: at 2 and 4 the
        # side share (1/P of the trailing update) is large enough that the cap
        # costs more than it saves -- one-rank-of-P replay, same box, two rounds:
        # P = 2 10.3-10.5 ms uncapped vs 11.5-11.8 capped, P = 4 8.1-8.7 vs 9.3,
        # P = 8 6.9-8.5 uncapped vs 6.8-7.1 at CUs - 16 (scripts/gpu_cap_by_p.sh, gpu_cap_p8.sh).
        self.side_cap = int(_native.lib().gelim_drbt_side_cap()) if self.gpu and self.P >= 8 else 0
        self.last_issue_s = None
        self._ud, self._vd = butterfly_diagonals(self.np, seed)
        lb = torch.arange(self.nloc) // NB
        self.gcol = ((lb * self.P + self.rank) * NB + torch.arange(self.nloc) % NB).to(self.device)
        self.last_steps, self.last_berr, self.last_fallback = 0, None, None
        self._plan = None
        self._fallback_solver = None
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        if self.fast:
            # the plan solves the ORIGINAL n-system (its refinement must not see the
            # identity padding) with the butterflies of order np (n padded to 128)
            lib = _native.lib()
            # GaussSolver's draw for the plan's own padding: the same butterflies,
            # so one rank reproduces the single-GPU hip-rbt solve bit for bit
            self._ud, self._vd = butterfly_diagonals(int(lib.gelim_mixed_padded(n)), seed)
            with torch.cuda.device(dev):
                self._plan = lib.gelim_mixed_plan_create2(n, self._ud.ctypes.data, self._vd.ctypes.data, 1)
            if not self._plan:
                raise _native.GelimError(_native.E_ARG, _native.last_error())
            return
        self.ud = torch.from_numpy(self._ud).to(dev)
        self.vd = torch.from_numpy(self._vd).to(dev)
        # column-block-major: slab lb = local block lb's np x 128 columns
        self.Mb = torch.zeros((self.nbl, self.np, NB), **f64)
        self.mbs = self.np * NB  # doubles between slabs
        self._Fs = self._Ds = None
        self._ain = torch.zeros(self.np, **f64)  # apply's input, captured by address
        nbuf = NBUF if lookahead else 2
        # landing buffers of the column messages [Dinv_k; L_k] (non-owners)
        self._xbufs = [torch.zeros(self.np * NB, **f64) for _ in range(nbuf)]
        self._Wm = torch.zeros((2, NB, NB), **f64)  # the native executor's W ring; the Python schedule uses [0]
        self._Ws = torch.zeros((NB, self.nloc), **f64)
        self._info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
        self._serr = torch.zeros(1, dtype=torch.int32, device=dev)  # block solves: hand-off timeout word
        if self.gpu:
            self._side = side_stream(dev)  # probed: never on the default stream's queue
        else:
            self._Wu = butterfly_dense(self._ud, self.np)
            Wv = butterfly_dense(self._vd, self.np)
            gc = self.gcol.cpu()
            self._Wv_loc = Wv[gc][:, gc].contiguous()
            self._Wv = Wv

    # -- data placement -------------------------------------------------------
    def empty_local(self) -> torch.Tensor:
        """np x ld storage: the rank's columns of the padded system, b (replicated) in column nloc."""
        return torch.zeros((self.np, self.ld), dtype=torch.float64, device=self.device)

    def _pad_identity(self, loc: torch.Tensor) -> None:
        pad = (self.gcol >= self.n).nonzero().flatten()
        if pad.numel():
            loc[self.gcol[pad], pad] = 1.0

    def scatter_from_global(self, aug: torch.Tensor) -> torch.Tensor:
        n = self.n
        loc = self.empty_local()
        real = (self.gcol < n).nonzero().flatten()
        loc[:n, real] = aug[:, :n].to(self.device)[:, self.gcol[real]]
        loc[:n, self.nloc] = aug[:, n].to(self.device)
        self._pad_identity(loc)
        return loc

    def generate_random(self, seed: int = 0) -> torch.Tensor:
        """The rank's columns of ops.init.random_system(n, seed) (bit-identical
        A) and b = A (1..n) by one all_reduce of the partial products."""
        n = self.n
        loc = self.empty_local()
        lib = _native.lib()
        for lb in range(self.nbl):
            g = lb * self.P + self.rank
            w = max(0, min(NB, n - g * NB))
            if w == 0:
                continue
            view = loc[:n, lb * NB:lb * NB + w]
            if self.gpu:
                _native.check(lib.gelim_gpu_init_random_block(ptr(view), loc.stride(0), 0, n, g * NB, w, seed,
                                                              stream_handle(self.device)), "init_random_block")
            else:
                tmp = torch.empty((n, w), dtype=torch.float64)
                lib.gelim_init_random_block_f64(ptr(tmp), w, 0, n, g * NB, w, seed)
                view.copy_(tmp)
        idx = torch.where(self.gcol < n, self.gcol + 1, torch.zeros_like(self.gcol)).to(torch.float64)
        b = loc[:, :self.nloc] @ idx
        self.comm.all_reduce(b)
        loc[:, self.nloc] = b
        self._pad_identity(loc)
        return loc

    # -- building blocks (HIP kernels on GPU ranks, torch on CPU ranks) ---------
    def _sh(self, stream=None):
        if not self.gpu:
            return None
        return stream.cuda_stream if stream is not None else stream_handle(self.device)

    def _transform(self, loc: torch.Tensor) -> None:
        if self.gpu:
            _native.check(_native.lib().gelim_drbt_transform(ptr(loc), self.ld, ptr(self.Mb), NB, self.mbs, self.np,
                                                             self.nloc, self.P, self.rank, ptr(self.ud), ptr(self.vd),
                                                             self._sh()), "drbt_transform")
        else:
            Mc = self._Wu.T @ loc[:, :self.nloc] @ self._Wv_loc
            self.Mb.copy_(Mc.view(self.np, self.nbl, NB).permute(1, 0, 2))

    def _col(self, k: int) -> torch.Tensor:
        """Column k from its diagonal block down, (np - 128 k) x 128, on this
        rank: the owner's slab, or the landing buffer of its message."""
        m = self.np - k * NB
        if k % self.P == self.rank:
            return self.Mb[k // self.P, k * NB:]
        return self._xbufs[k % len(self._xbufs)][:m * NB].view(m, NB)

    def _invert(self, k: int) -> None:
        """Owner of block k: Dinv_k = A_kk^-1 in place on the slab's diagonal
        block (kept there for the solves and sent as the head of column k)."""
        blk = self.Mb[k // self.P, k * NB:(k + 1) * NB]
        if self.gpu:
            _native.check(_native.lib().gelim_rbt_block_inverse(ptr(blk), NB, k * NB, ptr(blk), ptr(self._info),
                                                                self._sh()), "rbt_block_inverse")
        else:
            inv = torch.linalg.inv(blk)
            if not bool(torch.isfinite(inv).all()):
                self._info.fill_(min(int(self._info.item()), k * NB + 1))
            blk.copy_(inv)

    def _gemm_bm(self, C: torch.Tensor, cbm: bool, A: torch.Tensor, B: torch.Tensor, bbm: bool, ncols: int,
                 alpha: float, acc: bool, stream=None, cap: int = 0) -> None:
        """C (+)= alpha A B over ncols columns.  bbm / cbm: B / C is a run of
        column-block-major slabs starting at the given 2-D view (rows x 128
        each, slab stride mbs); otherwise a plain row-major 2-D view."""
        M_, K_ = A.shape[0], A.shape[1]
        if M_ == 0 or ncols == 0:
            return
        if self.gpu:
            _native.check(_native.lib().gelim_gpu_dgemm_bm(
                ptr(C), C.stride(0), self.mbs if cbm else 0, ptr(A), A.stride(0), ptr(B), B.stride(0),
                self.mbs if bbm else 0, M_, ncols, K_, alpha, int(acc), cap, self._sh(stream)), "dgemm_bm")
            return
        nbk = ncols // NB

        def slab(T: torch.Tensor, j: int, rows: int) -> torch.Tensor:  # block j of a slab run
            return T.as_strided((rows, NB), (T.stride(0), 1), T.storage_offset() + j * self.mbs)

        Bc = torch.cat([slab(B, j, K_) for j in range(nbk)], dim=1) if bbm else B[:, :ncols]
        prod = A @ Bc
        if alpha != 1.0:
            prod = prod * alpha
        if cbm:
            for j in range(nbk):
                Cj = slab(C, j, M_)
                if acc:
                    Cj.add_(prod[:, j * NB:(j + 1) * NB])
                else:
                    Cj.copy_(prod[:, j * NB:(j + 1) * NB])
        elif acc:
            C[:, :ncols].add_(prod)
        else:
            C[:, :ncols].copy_(prod)

    def _panel_w(self, k: int, col: torch.Tensor, lb0: int, lb1: int, W: torch.Tensor, stream=None,
                 cap: int = 0) -> None:
        """W[:, :128 (lb1 - lb0)] = Dinv_k M[k, local blocks lb0 .. lb1)."""
        if lb1 > lb0:
            self._gemm_bm(W, False, col[:NB], self.Mb[lb0, k * NB:(k + 1) * NB], True, (lb1 - lb0) * NB, 1.0,
                          False, stream, cap)

    def _panel_rows(self, k: int, col: torch.Tensor, lb0: int, lb1: int, r0: int, r1: int, W: torch.Tensor,
                    stream=None, cap: int = 0) -> None:
        """M[r0:r1, local blocks lb0 .. lb1) -= L_k[r0:r1] W (global rows
        r0 > 128 k; col row 0 is global row 128 k)."""
        if lb1 > lb0 and r1 > r0:
            self._gemm_bm(self.Mb[lb0, r0:r1], True, col[r0 - k * NB:r1 - k * NB], W, False, (lb1 - lb0) * NB,
                          -1.0, True, stream, cap)

    def _apply_panel(self, k: int, col: torch.Tensor, lb0: int, lb1: int, W: torch.Tensor, stream=None,
                     cap: int = 0) -> None:
        """Panel k applied to local blocks [lb0, lb1), every row below block k
        (cap > 0: the trailing GEMM on at most `cap` CUs)."""
        if lb1 > lb0:
            self._panel_w(k, col, lb0, lb1, W, stream)
            self._panel_rows(k, col, lb0, lb1, (k + 1) * NB, self.np, W, stream, cap)

    def _first_lb_after(self, k: int) -> int:
        """This rank's first local block with global index > k."""
        return min(self.nbl, max(0, -(-(k + 1 - self.rank) // self.P)))

    def _small(self, k: int) -> int:
        """Rows of the chain message of block k: Dinv_k and L_{k+1,k}."""
        return min(2 * NB, self.np - k * NB)

    # -- factorisation --------------------------------------------------------
    def factor_(self, loc: torch.Tensor) -> int:
        """Transform + block-LDU factorisation; returns 0 or 1 + the first
        column whose diagonal-block inverse is not finite (min over ranks)."""
        self._info.fill_(0x7F7F7F7F)
        self._transform(loc)
        if self.native_exec:
            t0 = time.perf_counter()
            self._factor_native()
            self.last_issue_s = time.perf_counter() - t0
        elif self.lookahead and self.gpu:
            t0 = time.perf_counter()
            self._replay("factor", self._factor_lookahead)
            self.last_issue_s = time.perf_counter() - t0  # host time to issue (or replay) the schedule
        else:
            self._factor_serial()
        v = self._info.to(torch.int64)
        self.comm.all_reduce(v, "min")
        val = int(self.comm.item(v))
        return 0 if val == 0x7F7F7F7F else val

    def _exec_args(self) -> _ExecArgs:
        a = _ExecArgs()
        a.np, a.nloc, a.P, a.rank = self.np, self.nloc, self.P, self.rank
        a.Mb, a.mbs = ptr(self.Mb), self.mbs
        for i, x in enumerate(self._xbufs):
            a.X[i] = ptr(x)
        a.Wm, a.Ws, a.info = ptr(self._Wm), ptr(self._Ws), ptr(self._info)
        a.main = torch.cuda.current_stream(self.device).cuda_stream
        a.side = self._side.cuda_stream
        a.comm = self.comm.comm_stream().cuda_stream
        if self.comm.native:
            a.rccl_small = self.comm.rccl_aux("small").handle
            a.rccl_bulk = self.comm.rccl().handle
        a.side_cap = self.side_cap
        return a

    def _factor_native(self) -> None:
        """The lookahead schedule of _factor_lookahead, issued by
        gelim_drbt_factor (csrc/hip/drbt_exec.hip): small messages on the
        main stream through a communicator of their own, bulk columns on the
        communicator stream through another."""
        lib = _native.lib()
        if self._exec is None:
            self._exec = lib.gelim_drbt_exec_create()
        a = self._exec_args()
        self._patch_exec_args(a)
        _native.check(lib.gelim_drbt_factor(self._exec, _C.byref(a)), "drbt_factor")

    def _patch_exec_args(self, a: _ExecArgs) -> None:
        """Hook (scripts/one_rank_of_p.py: the replay buffers)."""

    def _factor_serial(self) -> None:
        """One stream, one broadcast per block: the whole column message
        [Dinv_k; L_k], then every rank applies panel k to its later blocks."""
        comm, r, P = self.comm, self.rank, self.P
        for k in range(self.nb):
            o = k % P
            if r == o:
                self._invert(k)
            col = self._col(k)
            comm.broadcast(col.reshape(-1), src=o)
            self._apply_panel(k, col, self._first_lb_after(k), self.nbl, self._Ws)

    def _factor_lookahead(self) -> None:
        """Two streams, two broadcasts per block (module docstring).
          main (owner of k+1): [wait small_k] W = Dinv_k M[k, k+1];
               M[k+1, k+1] -= L_{k+1,k} W; invert it in place;
               [wait bulk_k] M[k+2.., k+1] -= L_{k+2..,k} W;
               broadcast small_{k+1}, bulk_{k+1}
          side (every rank): [wait small_k + bulk_k] panel k -> the next block
               this rank owns after k+1 (ev_first), then the rest (ev_rest)
        The chain (small_k -> two 128^3 GEMMs -> inverse) never waits for a
        bulk transfer unless that transfer is longer than the inverse."""
        comm, r, P, nb = self.comm, self.rank, self.P, self.nb
        main = torch.cuda.current_stream(self.device)
        side = self._side
        side.wait_stream(main)  # Mb as the transform left it
        nbuf = len(self._xbufs)
        ev_issue = [torch.cuda.Event() for _ in range(nb)]
        ev_first = [torch.cuda.Event() for _ in range(nb)]
        ev_rest = [torch.cuda.Event() for _ in range(nb)]
        hs, hb = {}, {}

        def ship(k: int) -> None:
            hs[k], hb[k] = self._ship(k)
            ev_issue[k].record(main)  # host-rendezvous transports land the data on main

        if r == 0:
            self._invert(0)
        else:
            self._foreign_chain(-1, None, None)
        ship(0)
        for k in range(nb):
            col = self._col(k)
            hs[k].wait()  # main: the chain message of block k
            side.wait_event(ev_issue[k])
            with torch.cuda.stream(side):
                hs[k].wait()  # side: all of column k
                if hb[k] is not None:
                    hb[k].wait()
                lb0 = self._first_lb_after(k)
                nxt = k + 1 < nb
                o1 = (k + 1) % P if nxt else -1
                ls = lb0 + (1 if o1 == r else 0)  # block k+1 is main's
                lf = min(ls + 1, self.nbl)
                self._apply_panel(k, col, ls, lf, self._Ws, side)
                ev_first[k].record(side)
                self._apply_panel(k, col, lf, self.nbl, self._Ws[:, (lf - ls) * NB:], side, self.side_cap)
                ev_rest[k].record(side)
            self._foreign_side(k, col, hs[k], hb[k])
            if not nxt:
                break
            if o1 == r:
                lb = lb0  # local block of k+1
                if k >= 1:
                    main.wait_event(ev_first[k - 1])  # panel k-1 reached block k+1 (side stream)
                self._panel_w(k, col, lb, lb + 1, self._Wm[0])
                self._panel_rows(k, col, lb, lb + 1, (k + 1) * NB, (k + 2) * NB, self._Wm[0])  # its diagonal block
                self._invert(k + 1)
                if hb[k] is not None:
                    hb[k].wait()  # main: L_{k+2.., k}
                    self._panel_rows(k, col, lb, lb + 1, (k + 2) * NB, self.np, self._Wm[0])
            else:
                self._foreign_chain(k, col, hb[k])
            if k + 1 >= nbuf:
                main.wait_event(ev_rest[k + 1 - nbuf])  # the landing buffer of k+1 is free again
            ship(k + 1)
        main.wait_event(ev_rest[nb - 1])

    def _ship(self, k: int):
        """Every rank: the two broadcasts of block k (the owner's slab in
        place): (handle of small_k, handle of bulk_k or None)."""
        o = k % self.P
        col = self._col(k).reshape(-1)
        sm = self._small(k) * NB
        hs = self.comm.broadcast_async(col[:sm], src=o)
        hb = self.comm.broadcast_async(col[sm:], src=o) if col.numel() > sm else None
        return hs, hb

    def _foreign_chain(self, k: int, col, hb) -> None:
        """Hook: the chain step that produces block k+1 runs on ANOTHER rank
        (nothing to do here; scripts/one_rank_of_p.py replays it on this GPU
        to measure one rank of a P-rank run)."""

    def _foreign_side(self, k: int, col, hs, hb) -> None:
        """Hook: panel k applied to block k+2 by ITS owner's side stream, when
        that owner is another rank (scripts/one_rank_of_p.py)."""

    # -- solves ----------------------------------------------------------------
    def _gather_solve_blocks(self) -> None:
        """All ranks get every super-diagonal S x S block of the factor and every
        diagonal-block inverse (one all_gather each)."""
        P, S, ns = self.P, NB * self.P, self.nbl
        mine = torch.empty((ns, S, NB), dtype=torch.float64, device=self.device)
        dmine = torch.empty((ns, NB, NB), dtype=torch.float64, device=self.device)
        for s in range(ns):
            mine[s] = self.Mb[s, s * S:(s + 1) * S]
            gb = s * P + self.rank  # global block of local block s: its inverse sits on its diagonal block
            dmine[s] = self.Mb[s, gb * NB:(gb + 1) * NB]
        g = torch.empty((P, ns, S, NB), dtype=torch.float64, device=self.device)
        self.comm.all_gather(g.view(-1), mine.view(-1))
        if getattr(self, "_Fs", None) is None:  # persistent: a captured apply reads them by address
            self._Fs = torch.empty((ns, S, S), dtype=torch.float64, device=self.device)
            self._Ds = torch.empty((ns, P, NB, NB), dtype=torch.float64, device=self.device)
        self._Fs.copy_(g.permute(1, 2, 0, 3).reshape(ns, S, S))
        gd = torch.empty((P, ns, NB, NB), dtype=torch.float64, device=self.device)
        self.comm.all_gather(gd.view(-1), dmine.view(-1))
        self._Ds.copy_(gd.permute(1, 0, 2, 3))  # (ns, P, 128, 128)
        del mine, dmine, g, gd

    def _super_solve(self, s: int, rhs: torch.Tensor, x: torch.Tensor, ysave: torch.Tensor | None,
                     upper: bool) -> None:
        P = self.P
        if self.gpu:
            # the single-GPU engine's persistent block solve (one workgroup per
            # 128-row block, hand-offs through sentinel-filled x): 12 us at
            # P = 8 against 190 us for the one-workgroup super_solve kernel
            # (profiles/dist_rbt_8rank_critical_path.md)
            _native.check(_native.lib().gelim_rbt_block_solve(ptr(self._Fs[s]), NB * P, ptr(self._Ds[s]), P, ptr(rhs),
                                                              ptr(x), ptr(ysave), int(upper), ptr(self._serr),
                                                              self._sh()), "rbt_block_solve")
            return
        F, D = self._Fs[s], self._Ds[s]
        order = reversed(range(P)) if upper else range(P)
        for b in order:
            R = slice(b * NB, (b + 1) * NB)
            C = slice((b + 1) * NB, P * NB) if upper else slice(0, b * NB)
            y = rhs[R] - F[R, C] @ x[C]
            if ysave is not None:
                ysave[R] = y
            x[R] = D[b] @ y

    def _gemv(self, A: torch.Tensor, x: torch.Tensor, y: torch.Tensor) -> None:
        """y += A x."""
        if A.shape[0] == 0:
            return
        if self.gpu:
            _native.check(_native.lib().gelim_drbt_gemv(ptr(A), A.stride(0), A.shape[0], A.shape[1], ptr(x), ptr(y),
                                                        1.0, self._sh()), "drbt_gemv")
        else:
            y += A @ x

    def _rbt_vec(self, v: torch.Tensor, d: torch.Tensor, transpose: bool, out: torch.Tensor) -> None:
        if self.gpu:
            _native.check(_native.lib().gelim_rbt_vec(ptr(v), 1, self.np, self.np, ptr(d), int(transpose), ptr(out),
                                                      self.np, self._sh()), "rbt_vec")
        else:
            W = self._Wu if transpose else self._Wv
            out.copy_(W.T @ v if transpose else W @ v)

    def _replay(self, name: str, fn):
        """fn() -- a fixed schedule over persistent buffers -- eagerly on its
        first call, then captured ONCE into a hipGraph (torch.cuda.graph: the
        side and communicator streams join the capture through their events,
        so the graph holds both streams' work and the RCCL collectives) and
        replayed on the current stream.  Returns fn's result (a static
        tensor of the graph when captured)."""
        if not self.graph:
            return fn()
        if name not in self._graphs:  # warm-up: RCCL / allocator first-call work stays out of the capture
            self._graphs[name] = None
            return fn()
        ent = self._graphs[name]
        if ent is None:
            g = torch.cuda.CUDAGraph()
            try:
                with self.comm.capturing(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                    out = fn()
            except Exception as e:  # noqa: BLE001 - a transport that cannot be captured: stay eager
                import warnings

                warnings.warn(f"DistributedRBT: hipGraph capture of {name} failed ({e!r}); issuing eagerly",
                              RuntimeWarning)
                self.graph = False
                torch.cuda.synchronize(self.device)
                return fn()
            ent = self._graphs[name] = (g, out)
        ent[0].replay()
        return ent[1]

    def apply(self, rhs: torch.Tensor) -> torch.Tensor:
        """(U^T)^-1-free correction: V (LU)^-1 U^T rhs for a replicated
        np-vector (graph-replayed on GPU ranks, see _replay)."""
        if not self.graph:
            return self._apply(rhs)
        self._ain.copy_(rhs)
        return self._replay("apply", lambda: self._apply(self._ain)).clone()

    def _apply(self, rhs: torch.Tensor) -> torch.Tensor:
        P, S, ns = self.P, NB * self.P, self.nbl
        r = self.rank
        dev = self.device
        c = torch.empty(self.np, dtype=torch.float64, device=dev)
        self._rbt_vec(rhs, self.ud if self.gpu else None, True, c)
        z = torch.empty_like(c)
        y = torch.empty_like(c)
        acc = torch.zeros_like(c)
        for s in range(ns):
            R = slice(s * S, (s + 1) * S)
            t = acc[R].clone()
            self.comm.all_reduce(t)
            self._super_solve(s, c[R] - t, z[R], y[R], False)
            if s + 1 < ns:
                zb = z[s * S + r * NB:s * S + (r + 1) * NB]
                self._gemv(self.Mb[s, (s + 1) * S:], zb, acc[(s + 1) * S:])
        xs = torch.empty_like(c)
        acc.zero_()
        for s in reversed(range(ns)):
            R = slice(s * S, (s + 1) * S)
            t = acc[R].clone()
            self.comm.all_reduce(t)
            self._super_solve(s, y[R] - t, xs[R], None, True)
            if s > 0:
                xb = xs[s * S + r * NB:s * S + (r + 1) * NB]
                self._gemv(self.Mb[s, :s * S], xb, acc[:s * S])
        out = torch.empty_like(c)
        self._rbt_vec(xs, self.vd if self.gpu else None, False, out)
        return out

    def _apply_timed_out(self) -> bool:
        """True on EVERY rank when any rank's block solves of the last apply
        timed out in a hand-off (its error word set; the result is then
        incomplete): one all_reduce max of the words, which are cleared.  All
        ranks then take the same fallback (the single-GPU engine's rule:
        gelim_mixed_solve hands such a system to partial pivoting) instead of
        one rank raising while the others block in the next collective."""
        v = self._serr.to(torch.int64)
        self.comm.all_reduce(v, "max")
        if int(self.comm.item(v)) == 0:
            return False
        self._serr.zero_()
        return True

    def _residual(self, loc: torch.Tensor, x: torch.Tensor) -> tuple[torch.Tensor, float]:
        """r = b - A x of the ORIGINAL n-system (x[n:] is zero: the identity
        padding is not part of the problem, as in gelim_mixed_solve) and the
        componentwise backward error max_{i<n} |r_i| / (|b| + |A||x|)_i (one
        all_reduce); r[n:] = 0."""
        xl = x[self.gcol].contiguous()
        yw = torch.empty((2, self.np), dtype=torch.float64, device=self.device)
        A = loc[:, :self.nloc]
        if self.gpu:
            _native.check(_native.lib().gelim_drbt_matvec_abs(ptr(loc), self.ld, self.np, self.nloc, ptr(xl),
                                                              ptr(yw[0]), ptr(yw[1]), self._sh()), "drbt_matvec_abs")
        else:
            yw[0] = A @ xl
            yw[1] = A.abs() @ xl.abs()
        self.comm.all_reduce(yw)
        n = self.n
        b = loc[:n, self.nloc]
        r = torch.zeros(self.np, dtype=torch.float64, device=self.device)
        r[:n] = b - yw[0, :n]
        w = b.abs() + yw[1, :n]
        tiny = torch.finfo(torch.float64).tiny
        rn = r[:n]
        om = torch.where(w > 0, rn.abs() / w.clamp_min(tiny), torch.where(rn != 0, torch.full_like(rn, math.inf), rn))
        return r, float(self.comm.item(om.max()))

    # -- the solve --------------------------------------------------------------
    def solve_(self, loc: torch.Tensor) -> torch.Tensor:
        """x (n entries, replicated on every rank) of the local system `loc`
        (np x ld from generate_random / scatter_from_global; kept intact, it is
        the residual's system)."""
        self.last_steps, self.last_berr, self.last_fallback = 0, None, None
        if self.fast:
            return self._solve_single(loc)
        info = self.factor_(loc)
        if info:
            return self._fallback(loc, f"no-pivot LU: non-finite diagonal-block inverse at column {info - 1}")
        self._gather_solve_blocks()
        x = self.apply(loc[:, self.nloc].contiguous())
        if self._apply_timed_out():
            return self._fallback(loc, "block-solve hand-off timed out")
        x[self.n:] = 0.0
        eps = torch.finfo(torch.float64).eps
        strict, loose = 4.0 * eps, max(math.sqrt(self.n), 8.0) * eps
        prev, best, xb = math.inf, math.inf, None
        for it in range(self.max_steps + 1):
            r, om = self._residual(loc, x)
            self.last_steps, self.last_berr = it, om
            if om <= strict:
                return x[:self.n]
            if not om < 0.9 * prev or it == self.max_steps:  # NaN, stagnated or out of steps
                if om <= loose and om <= best:
                    return x[:self.n]
                if best <= loose:
                    self.last_berr = best
                    return xb[:self.n]
                return self._fallback(loc, f"refinement stalled after {it} corrections (componentwise backward "
                                           f"error {om:.3e})")
            if om < best:
                best, xb = om, x.clone()
            prev = om
            x = x + self.apply(r)
            if self._apply_timed_out():
                return self._fallback(loc, "block-solve hand-off timed out")
            x[self.n:] = 0.0
        raise AssertionError("unreachable")

    def _solve_single(self, loc: torch.Tensor) -> torch.Tensor:
        """One rank: the native single-GPU solve of the padded augmented system."""
        import ctypes

        n = self.n
        if n == self.np:  # the local storage is the augmented system [A | b]
            aug, ld = loc, self.ld
        else:  # b sits at column np: an (n, n+1) copy for the native solve
            aug = torch.empty((n, n + 2), dtype=torch.float64, device=self.device)
            aug[:, :n] = loc[:n, :n]
            aug[:, n] = loc[:n, self.nloc]
            ld = n + 2
        x = torch.empty(n, dtype=torch.float64, device=self.device)
        st, be = ctypes.c_int(0), ctypes.c_double(0.0)
        rc = _native.check(_native.lib().gelim_mixed_solve(self._plan, ptr(aug), ld, ptr(x), self.max_steps,
                                                           ctypes.byref(st), ctypes.byref(be), self._sh()),
                           "mixed_solve")
        self.last_steps, self.last_berr = st.value, be.value
        if rc == 1:
            return self._fallback(loc, f"no-pivot LU: zero pivot or refinement stalled after {st.value} corrections")
        return x

    def _fallback(self, loc: torch.Tensor, reason: str) -> torch.Tensor:
        """Partial pivoting (DistributedGauss) on the same system: its
        128-column block layout puts block g on rank g % P at the same local
        column, so the slab is a copy of ours."""
        from .dist_gauss import DistributedGauss

        self.last_fallback = reason
        if self._fallback_solver is None:
            self._fallback_solver = DistributedGauss(self.comm, self.n, block=NB)
        dg = self._fallback_solver
        gl = dg.empty_local()
        rows = min(dg.n_pad, self.np)
        w = min(dg.nloc, self.nloc)
        gl[:rows, :w] = loc[:rows, :w]
        gl[:rows, dg.nloc] = loc[:rows, self.nloc]
        return dg.solve_(gl)

    def close(self) -> None:
        if self._plan:
            _native.lib().gelim_mixed_plan_destroy(self._plan)
            self._plan = None
        if getattr(self, "_exec", None):
            if self.gpu:
                torch.cuda.synchronize(self.device)  # its events may still be in flight
            _native.lib().gelim_drbt_exec_destroy(self._exec)
            self._exec = None
