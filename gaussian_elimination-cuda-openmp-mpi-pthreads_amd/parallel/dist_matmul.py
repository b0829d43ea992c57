"""Distributed fp32 matrix multiply C = A @ B across GPUs (RCCL).

The reference has no distributed matmul; BASELINE.json asks for a 16384^2
fp32 multiply across the 8 GPUs of one node.  Two decompositions:

allgather_matmul (1-D, default)
  A and C row-partitioned, B row-partitioned into P k-blocks.  B is gathered
  in column chunks with all_gather_into_tensor -- one RCCL collective per
  chunk, which spreads over every xGMI link of the node (the ring below
  drives ONE neighbour link per step).  The rank's own k-block needs no
  communication, so C = A_loc[:, own] @ B_loc runs first, under the first
  chunk's gather; then chunk c+1's gather runs on the RCCL stream while the
  MFMA GEMM adds the other ranks' k-blocks of chunk c.

ring_matmul (1-D)
  A and C row-partitioned, B row-partitioned into P k-blocks.  P steps: each
  rank multiplies its A slice against the B block it currently holds
  (accumulating into C with the MFMA kernel) while that block is passed to
  the next rank with one batched isend/irecv on the communication stream — i.e. an
  all-gather of B overlapped with compute, never materialising B whole.
  Per step each GPU sends/receives one K/P x N block over one xGMI link.

summa_matmul (2-D, pr x pc grid)
  A (M/pr x K/pc) and B (K/pr x N/pc) blocks; for each k-panel (a multiple
  of lcm(pr, pc) of them) the owning column broadcasts its A panel along the
  process row and the owning row its B panel along the process column, then
  every rank accumulates its C block.  Row/column sub-communicators; the
  broadcasts are asynchronous into double buffers, so panel l+1 travels
  while panel l multiplies.

Compute runs on the native kernels (`gelim_gpu_matmul_f32_ex`, accumulate
mode); on CPU ranks (gloo tests) the accumulate is torch.addmm.
"""
from __future__ import annotations

import math

import torch

from .. import _native
from ..ops.matmul import KERNELS
from ..utils.tensors import ptr, row_major_ld, stream_handle
from .comm import Communicator


def matmul_acc_(C: torch.Tensor, A: torch.Tensor, B: torch.Tensor, accumulate: bool, kernel: str = "mfma") -> None:
    """C (+)= A @ B on strided row-major views."""
    M, K = A.shape
    N = B.shape[1]
    if C.device.type == "cuda":
        _native.check(_native.lib().gelim_gpu_matmul_f32_ex(
            ptr(A), row_major_ld(A), ptr(B), row_major_ld(B), ptr(C), row_major_ld(C), M, N, K,
            int(accumulate), KERNELS[kernel], stream_handle(C.device)), "matmul_f32_ex")
    elif accumulate:
        C.addmm_(A, B)
    else:
        torch.mm(A, B, out=C)


def ring_matmul(comm: Communicator, A_loc: torch.Tensor, B_loc: torch.Tensor, kernel: str = "mfma"
                ) -> torch.Tensor:
    """A_loc: (M/P, K) rows of A; B_loc: (K/P, N) rows of B (equal blocks).
    Returns C_loc = A_loc @ B (M/P, N)."""
    P, r = comm.world_size, comm.rank
    kb, N = B_loc.shape
    if A_loc.shape[1] != kb * P:
        raise ValueError("ring_matmul needs K divisible by the world size")
    C = torch.empty((A_loc.shape[0], N), dtype=torch.float32, device=A_loc.device)
    cur = B_loc.contiguous()
    # receive buffers: the caller's B_loc is only ever read (it may be a view
    # of a larger tensor), so the ring rotates through two scratch blocks
    bufs = [torch.empty_like(cur) for _ in range(min(2, P - 1))]
    for t in range(P):
        src = (r - t) % P  # whose B block we hold now
        reqs = []
        nxt = bufs[t % 2] if t < P - 1 else None
        if t < P - 1:
            reqs = comm.sendrecv(cur, (r + 1) % P, nxt, (r - 1) % P)
        matmul_acc_(C, A_loc[:, src * kb:(src + 1) * kb], cur, accumulate=t > 0, kernel=kernel)
        for q in reqs:
            q.wait()
        if t < P - 1:
            # the send of `cur` has completed (waited) before its buffer is
            # received into again two steps later
            cur = nxt
    return C


def default_chunks(P: int) -> int:
    """Column chunks of the allgather: enough to hide each gather under the
    previous chunk's GEMM, few enough that each GEMM still fills the GPU."""
    return 2 if P <= 2 else 4


def allgather_matmul(comm: Communicator, A_loc: torch.Tensor, B_loc: torch.Tensor, chunks: int | None = None,
                     kernel: str = "mfma") -> torch.Tensor:
    """A_loc: (M/P, K) rows of A; B_loc: (K/P, N) rows of B (equal blocks,
    rank order).  Returns C_loc = A_loc @ B (M/P, N).  B travels as `chunks`
    column chunks, each gathered (async) while the previous one multiplies;
    the rank's own k-block multiplies under the first gather."""
    P, r = comm.world_size, comm.rank
    kb, N = B_loc.shape
    if A_loc.shape[1] != kb * P:
        raise ValueError("allgather_matmul needs K divisible by the world size")
    C = torch.empty((A_loc.shape[0], N), dtype=torch.float32, device=A_loc.device)
    if P == 1 and not comm.distributed:  # (a one-rank process group still runs the gathers)
        matmul_acc_(C, A_loc, B_loc, accumulate=False, kernel=kernel)
        return C
    chunks = max(1, min(chunks or default_chunks(P), N))
    bounds = [N * c // chunks for c in range(chunks + 1)]
    wmax = max(bounds[c + 1] - bounds[c] for c in range(chunks))
    send = [torch.empty((kb, wmax), dtype=torch.float32, device=A_loc.device) for _ in range(2)]
    recv = [torch.empty((P * kb, wmax), dtype=torch.float32, device=A_loc.device) for _ in range(2)]

    def post(c: int):
        w = bounds[c + 1] - bounds[c]
        snd = send[c % 2][:, :w]
        snd.copy_(B_loc[:, bounds[c]:bounds[c + 1]])
        out = recv[c % 2].view(-1)[:P * kb * w]
        return comm.all_gather_async(out, snd.contiguous()), out.view(P * kb, w)

    pending = post(0)
    # own k-block: no communication needed, runs under the first gather
    matmul_acc_(C, A_loc[:, r * kb:(r + 1) * kb], B_loc, accumulate=False, kernel=kernel)
    for c in range(chunks):
        h, Bc = pending
        h.wait()
        if c + 1 < chunks:
            pending = post(c + 1)  # on the RCCL stream while chunk c multiplies
        Cc = C[:, bounds[c]:bounds[c + 1]]
        if r > 0:
            matmul_acc_(Cc, A_loc[:, :r * kb], Bc[:r * kb], accumulate=True, kernel=kernel)
        if r < P - 1:
            matmul_acc_(Cc, A_loc[:, (r + 1) * kb:], Bc[(r + 1) * kb:], accumulate=True, kernel=kernel)
    return C


def grid_shape(P: int) -> tuple[int, int]:
    """Most square pr x pc factorisation with pr <= pc."""
    pr = int(math.isqrt(P))
    while P % pr:
        pr -= 1
    return pr, P // pr


def summa_matmul(comm: Communicator, A_blk: torch.Tensor, B_blk: torch.Tensor, grid: tuple[int, int] | None = None,
                 kernel: str = "mfma", groups: tuple | None = None, panels: int | None = None) -> torch.Tensor:
    """A_blk: block (i, j) of A (M/pr x K/pc); B_blk: block (i, j) of B
    (K/pr x N/pc); rank = i*pc + j.  Returns C block (i, j).  panels: number
    of k-panels (a multiple of lcm(pr, pc) dividing K; default: lcm(pr, pc)
    split further until a panel is <= 1024 deep, for overlap)."""
    P, r = comm.world_size, comm.rank
    pr, pc = grid or grid_shape(P)
    if pr * pc != P:
        raise ValueError("grid does not match the world size")
    i, j = divmod(r, pc)
    row_comm, col_comm = groups or make_summa_groups(comm, pr, pc)
    mb, ka = A_blk.shape
    kb_rows, nb = B_blk.shape
    K = ka * pc
    if kb_rows * pr != K:
        raise ValueError("inconsistent K split")
    base = pr * pc // math.gcd(pr, pc)
    if panels is None:
        panels = base
        while K // panels > 1024 and K % (panels * 2) == 0:
            panels *= 2
    if panels % base or K % panels:
        raise ValueError(f"panels must be a multiple of {base} dividing K={K}")
    Lp = panels
    kp = K // Lp
    dev = A_blk.device
    C = torch.empty((mb, nb), dtype=torch.float32, device=dev)
    a_pan = [torch.empty((mb, kp), dtype=torch.float32, device=dev) for _ in range(2)]
    b_pan = [torch.empty((kp, nb), dtype=torch.float32, device=dev) for _ in range(2)]

    def post(l: int):
        """Panel l into buffer l % 2: copies and broadcasts enqueued after the
        GEMM of panel l-2 (stream order), so its buffer is free."""
        k0 = l * kp
        ja, off_a = divmod(k0, ka)  # process column owning this A panel
        ib, off_b = divmod(k0, kb_rows)  # process row owning this B panel
        if j == ja:
            a_pan[l % 2].copy_(A_blk[:, off_a:off_a + kp])
        ha = row_comm.broadcast_async(a_pan[l % 2], src=ja)
        if i == ib:
            b_pan[l % 2].copy_(B_blk[off_b:off_b + kp, :])
        hb = col_comm.broadcast_async(b_pan[l % 2], src=ib)
        return ha, hb

    pending = post(0)
    for l in range(Lp):
        ha, hb = pending
        ha.wait()
        hb.wait()
        if l + 1 < Lp:
            pending = post(l + 1)  # travels while panel l multiplies
        matmul_acc_(C, a_pan[l % 2], b_pan[l % 2], accumulate=l > 0, kernel=kernel)
    return C


def make_summa_groups(comm: Communicator, pr: int, pc: int):
    """Row and column sub-communicators (every rank creates every group)."""
    row_comm = col_comm = None
    i, j = divmod(comm.rank, pc)
    for a in range(pr):
        g = comm.subgroup([a * pc + b for b in range(pc)])
        if a == i:
            row_comm = g
    for b in range(pc):
        g = comm.subgroup([a * pc + b for a in range(pr)])
        if b == j:
            col_comm = g
    return row_comm, col_comm
