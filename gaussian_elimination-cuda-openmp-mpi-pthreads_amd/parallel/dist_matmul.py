"""Distributed fp32 matrix multiply C = A @ B across GPUs (RCCL).

The reference has no distributed matmul; BASELINE.json asks for a 16384^2
fp32 multiply across the 8 GPUs of one node.  Two decompositions:

allgather_matmul (1-D, default)
  A and C row-partitioned, B row-partitioned into P k-blocks.  B is gathered
  in column chunks with all_gather_into_tensor -- one RCCL collective per
  chunk, which spreads over every xGMI link of the node (the ring below
  drives ONE neighbour link per step) -- and chunk c+1's gather runs on the
  RCCL stream while the MFMA GEMM computes C[:, chunk c] = A_loc @ B[:, c].

ring_matmul (1-D)
  A and C row-partitioned, B row-partitioned into P k-blocks.  P steps: each
  rank multiplies its A slice against the B block it currently holds
  (accumulating into C with the MFMA kernel) while that block is passed to
  the next rank with one batched isend/irecv on the communication stream — i.e. an
  all-gather of B overlapped with compute, never materialising B whole.
  Per step each GPU sends/receives one K/P x N block over one xGMI link.

summa_matmul (2-D, pr x pc grid)
  A (M/pr x K/pc) and B (K/pr x N/pc) blocks; for each of lcm(pr,pc)
  k-panels the owning column broadcasts its A panel along the process row
  and the owning row its B panel along the process column, then every rank
  accumulates its C block.  Uses row/column sub-communicators.

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


def allgather_matmul(comm: Communicator, A_loc: torch.Tensor, B_loc: torch.Tensor, chunks: int = 4,
                     kernel: str = "mfma") -> torch.Tensor:
    """A_loc: (M/P, K) rows of A; B_loc: (K/P, N) rows of B (equal blocks,
    rank order).  Returns C_loc = A_loc @ B (M/P, N).  B travels as `chunks`
    column chunks, each gathered (async) while the previous one multiplies."""
    P = comm.world_size
    kb, N = B_loc.shape
    if A_loc.shape[1] != kb * P:
        raise ValueError("allgather_matmul needs K divisible by the world size")
    C = torch.empty((A_loc.shape[0], N), dtype=torch.float32, device=A_loc.device)
    if P == 1:
        matmul_acc_(C, A_loc, B_loc, accumulate=False, kernel=kernel)
        return C
    chunks = max(1, min(chunks, N))
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
    for c in range(chunks):
        h, Bc = pending
        h.wait()
        if c + 1 < chunks:
            pending = post(c + 1)  # on the RCCL stream while chunk c multiplies
        matmul_acc_(C[:, bounds[c]:bounds[c + 1]], A_loc, Bc, accumulate=False, kernel=kernel)
    return C


def grid_shape(P: int) -> tuple[int, int]:
    """Most square pr x pc factorisation with pr <= pc."""
    pr = int(math.isqrt(P))
    while P % pr:
        pr -= 1
    return pr, P // pr


def summa_matmul(comm: Communicator, A_blk: torch.Tensor, B_blk: torch.Tensor, grid: tuple[int, int] | None = None,
                 kernel: str = "mfma", groups: tuple | None = None) -> torch.Tensor:
    """A_blk: block (i, j) of A (M/pr x K/pc); B_blk: block (i, j) of B
    (K/pr x N/pc); rank = i*pc + j.  Returns C block (i, j)."""
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
    Lp = pr * pc // math.gcd(pr, pc)  # number of k-panels
    kp = K // Lp
    C = torch.empty((mb, nb), dtype=torch.float32, device=A_blk.device)
    a_pan = torch.empty((mb, kp), dtype=torch.float32, device=A_blk.device)
    b_pan = torch.empty((kp, nb), dtype=torch.float32, device=A_blk.device)
    for l in range(Lp):
        k0 = l * kp
        ja, off_a = divmod(k0, ka)  # process column owning this A panel
        ib, off_b = divmod(k0, kb_rows)  # process row owning this B panel
        if j == ja:
            a_pan.copy_(A_blk[:, off_a:off_a + kp])
        row_comm.broadcast(a_pan, src=ja)
        if i == ib:
            b_pan.copy_(B_blk[off_b:off_b + kp, :])
        col_comm.broadcast(b_pan, src=ib)
        matmul_acc_(C, a_pan, b_pan, accumulate=l > 0, kernel=kernel)
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
