"""Communicator layer (L4 of SURVEY.md §1) — replaces the reference's MPI.

One process per GPU, `torch.distributed` underneath: backend "nccl" is RCCL
on ROCm (collectives over xGMI), "gloo" is the CPU transport used for tests
and for CPU-only ranks.  The reference's MPI call sites map as
(SURVEY.md §2.5):

  MPI_Init/Comm_size/Comm_rank/Finalize  -> init_from_env / destroy
  MPI_Bcast(pivot row)                    -> broadcast (one PANEL per call)
  MPI_Send/Isend/Recv/Irecv row blocks    -> none: data stays resident,
                                             owner-computes
  MPI_Barrier                             -> barrier (stream-ordered otherwise)
  (solution assembly)                     -> all_reduce / all_gather

Rendezvous always uses 127.0.0.1 defaults (the container hostname may not
resolve).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


class _Done:
    """Handle of a collective that needed no communication."""

    def wait(self) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


class _Staged:
    """Handle of a point-to-point op staged through host memory: wait()
    completes the host transfer, then copies a received buffer to the
    device tensor."""

    def __init__(self, work, host: torch.Tensor, dst: torch.Tensor | None = None):
        self.work, self.host, self.dst = work, host, dst

    def wait(self) -> bool:
        self.work.wait()
        if self.dst is not None:
            self.dst.copy_(self.host)
        return True

    def is_completed(self) -> bool:
        return self.work.is_completed()


class _Event:
    """Handle of a collective issued on the communicator's own stream:
    wait() makes the CURRENT stream wait for it (no host block)."""

    def __init__(self, ev: torch.cuda.Event):
        self.ev = ev

    def wait(self) -> bool:
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self) -> bool:
        return self.ev.query()


@dataclass
class Communicator:
    rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    backend: str = "none"
    group: object = None
    # a torch.distributed group is live even at ONE rank (init_from_env
    # force_pg / GELIM_FORCE_PG=1): every collective then really goes through
    # the backend (RCCL on a GPU), which is how the RCCL path of every
    # distributed schedule is exercised on a one-GPU box
    pg: bool = False
    _cstream: object = field(default=None, repr=False, compare=False)

    # -- collectives ------------------------------------------------------
    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.pg

    @property
    def own_stream(self) -> bool:
        """RCCL ranks issue their asynchronous collectives on a dedicated,
        probed stream (comm_stream) rather than on torch's internal RCCL
        stream, a pool stream whose hardware queue nobody checks: HIP maps
        streams onto GPU_MAX_HW_QUEUES (4) queues, and a collective whose
        queue is the lookahead side stream's would wait behind the whole
        trailing update (profiles/hw_queues_r4.txt).  GELIM_COMM_STREAM=torch
        restores torch's own stream (A/B)."""
        return (self.backend == "nccl" and self.device.type == "cuda"
                and os.environ.get("GELIM_COMM_STREAM", "own") != "torch")

    def comm_stream(self) -> torch.cuda.Stream:
        """The stream this rank's asynchronous collectives run on: a
        process-lifetime stream on a hardware queue of its own, probed to run
        beside the default stream and the lookahead side stream
        (utils/tensors.dedicated_stream).  A synchronous collective
        (async_op=False) runs on the CURRENT stream in torch >= 2.7, so it is
        issued under this stream."""
        if self._cstream is None:
            from ..utils.tensors import dedicated_stream

            self._cstream = dedicated_stream(self.device, "comm")
        return self._cstream

    def _on_comm_stream(self, issue) -> _Event:
        cs = self.comm_stream()
        cs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cs):
            issue()
            ev = torch.cuda.Event()
            ev.record(cs)
        return _Event(ev)

    @property
    def staged(self) -> bool:
        """gloo ranks holding device tensors (several ranks sharing one GPU,
        which RCCL refuses): broadcast and all_reduce use gloo's own device
        path (asynchronous, stream-ordered); all_gather and point-to-point
        ops, which it lacks for device tensors, go through host memory."""
        return self.backend == "gloo" and self.device.type == "cuda"

    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self.distributed:
            dist.broadcast(t, src=self.global_rank(src), group=self.group)
        return t

    def broadcast_async(self, t: torch.Tensor, src: int):
        """Non-blocking broadcast: returns a handle whose wait() makes the
        current stream wait for the data (RCCL runs on its own stream, after
        the work already queued on the current one)."""
        if self.distributed and self.own_stream:
            return self._on_comm_stream(lambda: dist.broadcast(t, src=self.global_rank(src), group=self.group))
        if self.distributed:
            return dist.broadcast(t, src=self.global_rank(src), group=self.group, async_op=True)
        return _Done()

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.distributed:
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=self.group)
        return t

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """out: (world_size * t.numel()) contiguous tensor."""
        if self.distributed and self.staged:
            ho = torch.empty(out.numel(), dtype=out.dtype)
            dist.all_gather_into_tensor(ho, t.detach().reshape(-1).cpu(), group=self.group)
            out.view(-1).copy_(ho)
        elif self.distributed:
            dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        else:
            out.view(-1).copy_(t.reshape(-1))
        return out

    def all_gather_async(self, out: torch.Tensor, t: torch.Tensor):
        """Non-blocking all_gather_into_tensor (see broadcast_async); staged
        ranks complete it before returning."""
        if self.distributed and self.staged:
            self.all_gather(out, t)
            return _Done()
        if self.distributed and self.own_stream:
            src = t.contiguous().view(-1)
            return self._on_comm_stream(lambda: dist.all_gather_into_tensor(out.view(-1), src, group=self.group))
        if self.distributed:
            return dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1), group=self.group,
                                               async_op=True)
        out.view(-1).copy_(t.reshape(-1))
        return _Done()

    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def send(self, t: torch.Tensor, dst: int):
        if self.staged:
            h = t.detach().cpu()
            return _Staged(dist.isend(h, dst=self.global_rank(dst), group=self.group), h)
        return dist.isend(t, dst=self.global_rank(dst), group=self.group)

    def recv(self, t: torch.Tensor, src: int):
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            return _Staged(dist.irecv(h, src=self.global_rank(src), group=self.group), h, t)
        return dist.irecv(t, src=self.global_rank(src), group=self.group)

    def sendrecv(self, send_t: torch.Tensor, dst: int, recv_t: torch.Tensor, src: int) -> list:
        """Send to dst and receive from src as ONE batched p2p operation
        (batch_isend_irecv: RCCL group semantics, so a ring of such calls
        cannot deadlock on serialised send kernels).  Returns the requests."""
        if self.staged:
            hs = send_t.detach().cpu()
            hr = torch.empty(recv_t.shape, dtype=recv_t.dtype)
            ops = [dist.P2POp(dist.isend, hs, self.global_rank(dst), self.group),
                   dist.P2POp(dist.irecv, hr, self.global_rank(src), self.group)]
            works = dist.batch_isend_irecv(ops)
            return [_Staged(works[0], hs), _Staged(works[1], hr, recv_t)]
        ops = [dist.P2POp(dist.isend, send_t, self.global_rank(dst), self.group),
               dist.P2POp(dist.irecv, recv_t, self.global_rank(src), self.group)]
        return dist.batch_isend_irecv(ops)

    def global_rank(self, r: int) -> int:
        if self.group is None:
            return r
        return dist.get_global_rank(self.group, r)

    def subgroup(self, ranks: list[int]) -> "Communicator":
        """Communicator over a subset of ranks (SUMMA rows/columns).  Must be
        called by every rank with the same list (torch requirement)."""
        if not self.distributed:  # one rank: the only subgroup is itself
            return Communicator(0, 1, self.device, self.backend, None)
        g = dist.new_group(ranks=ranks, backend=self.backend if self.backend != "none" else None)
        if self.rank not in ranks:
            return Communicator(0, 1, self.device, self.backend, None)
        return Communicator(ranks.index(self.rank), len(ranks), self.device, self.backend, g,
                            pg=self.pg, _cstream=self._cstream)

    def overlap_probe(self, other: torch.cuda.Stream, ticks: int = 500000) -> bool:
        """True when an asynchronous collective (broadcast_async) plus the
        current stream's wait on it do NOT queue behind a kernel running on
        `other` (the lookahead side stream): a bounded waiter kernel (5 ms)
        runs on `other` until a setter kernel, queued on the current stream
        after the broadcast, releases it.  False means the collective or the
        current stream shares `other`'s hardware queue -- the lookahead would
        silently serialise."""
        from .. import _native
        from ..utils.tensors import ptr

        lib = _native.lib()
        dev = self.device
        words = torch.zeros(2, dtype=torch.int32, device=dev)
        t = torch.zeros(4096, dtype=torch.float64, device=dev)
        # warm-up first: the stream set-up (probes that synchronise streams)
        # and the collective's first-call work must not run under the waiter
        self.broadcast_async(t, 0).wait()
        torch.cuda.synchronize(dev)
        _native.check(lib.gelim_gpu_probe_kernel(other.cuda_stream, ptr(words), 0, ticks), "probe_kernel")
        self.broadcast_async(t, 0).wait()
        _native.check(lib.gelim_gpu_probe_kernel(torch.cuda.current_stream(dev).cuda_stream, ptr(words), 1, 0),
                      "probe_kernel")
        torch.cuda.synchronize(dev)
        return int(words[1].item()) == 1


def env_world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init_from_env(backend: str | None = None, device: str | None = None,
                  timeout_s: float = 600.0, force_pg: bool | None = None) -> Communicator:
    """Join the job described by RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* (torchrun).
    backend None -> GELIM_DIST_BACKEND if set, else "nccl" (RCCL) when a GPU
    is visible, else "gloo".  gloo with a GPU device is the transport of
    several ranks sharing ONE GPU (tests): device tensors, host-staged where
    gloo has no device path (Communicator.staged).

    force_pg (default: GELIM_FORCE_PG=1): a one-rank job still creates the
    process group (an in-memory store, no rendezvous), so the distributed
    schedules run their collectives through RCCL on a single GPU."""
    rank, world, local = env_world()
    use_gpu = device != "cpu" and (device is not None or torch.cuda.is_available())
    want = backend or os.environ.get("GELIM_DIST_BACKEND")
    if use_gpu:
        # one rank per GPU; over gloo, more ranks than GPUs share them round-robin
        ndev = max(1, torch.cuda.device_count())
        idx = local % ndev if want == "gloo" else local
        dev = torch.device(device) if device not in (None, "cuda") else torch.device("cuda", idx)
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if force_pg is None:
        force_pg = os.environ.get("GELIM_FORCE_PG", "0") == "1"
    if world <= 1 and not force_pg:
        return Communicator(0, 1, dev, "none")
    if world <= 1:
        backend = backend or os.environ.get("GELIM_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        if not dist.is_initialized():
            kw = dict(backend=backend, store=dist.HashStore(), rank=0, world_size=1,
                      timeout=datetime.timedelta(seconds=timeout_s))
            if backend == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(**kw)
        return Communicator(0, 1, dev, backend, pg=True)
    backend = backend or os.environ.get("GELIM_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
    # failure detection: a rank that dies or hangs must not leave the others
    # blocked forever.  RCCL's async error handling turns a collective that
    # exceeds `timeout_s` (or a communicator error) into an abort + host
    # exception on every surviving rank; gloo raises on the same timeout.
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return Communicator(rank, world, dev, backend)


def destroy() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
