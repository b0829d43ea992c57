"""In-process emulated communicator: P ranks as P threads of ONE process, all
on one device ("Distributed (emulated)").

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), and the GPU
boxes this framework is tested on expose a single MI355X, so the distributed
algorithms (column block-cyclic Gauss, ring / SUMMA matmul) need a transport
that runs P ranks against one card with the SAME collective semantics as
`Communicator` (broadcast / all_reduce / all_gather / barrier / isend-irecv /
subgroups).  Each rank is a Python thread; collectives meet at a
`threading.Barrier` and exchange tensors through shared slots:

  broadcast   src posts its tensor, everyone else copies it
  all_reduce  every rank reduces ALL slots in rank order (deterministic, so
              every rank gets a bit-identical result, like a ring all-reduce
              with a fixed order would)
  all_gather  concatenation of the slots in rank order
  send/recv   per-(src, dst) FIFO mailboxes; recv's wait() copies

Device ordering: the threads issue on their thread's current stream (the
default stream unless a test sets one), so a copy of another rank's tensor
is enqueued after that rank enqueued its producer and before it enqueues any
overwrite (which only happens after the closing barrier).  The HIP kernels
release the GIL (ctypes / torch), so the ranks' host code genuinely
interleaves, like P processes would.

Failures: a rank that raises aborts the world barrier, so the other ranks
get `BrokenBarrierError` instead of hanging (the emulated analogue of RCCL's
async-error abort); `run_emulated` re-raises the first rank's exception.
"""
from __future__ import annotations

import queue
import threading
from typing import Any, Callable

import torch

from .comm import Communicator


class _World:
    def __init__(self, size: int, timeout_s: float):
        self.size = size
        self.timeout_s = timeout_s
        self.barrier = threading.Barrier(size)
        self.slots: list[Any] = [None] * size
        self.mail: dict[tuple[int, int], queue.Queue] = {}
        self.lock = threading.Lock()
        self.subworlds: dict[tuple, list] = {}

    def box(self, src: int, dst: int) -> queue.Queue:
        with self.lock:
            return self.mail.setdefault((src, dst), queue.Queue())

    def wait(self) -> None:
        self.barrier.wait(self.timeout_s)

    def abort(self) -> None:
        self.barrier.abort()
        with self.lock:
            subs = [w for ws in self.subworlds.values() for w in ws if isinstance(w, _World)]
        for w in subs:
            w.abort()


class _Done:
    def wait(self) -> bool:
        return True

    def is_completed(self) -> bool:
        return True


class _RecvReq:
    def __init__(self, box: queue.Queue, out: torch.Tensor, timeout_s: float):
        self.box, self.out, self.timeout_s, self.done = box, out, timeout_s, False

    def wait(self) -> bool:
        if not self.done:
            self.out.copy_(self.box.get(timeout=self.timeout_s))
            self.done = True
        return True

    def is_completed(self) -> bool:
        return self.done


class EmulatedComm(Communicator):
    """One rank of an in-process emulated world (see module docstring)."""

    def __init__(self, world: _World, rank: int, device: torch.device):
        super().__init__(rank=rank, world_size=world.size, device=device, backend="emulated", group=None)
        self._w = world

    # every collective is two barriers: post -> (read) -> release
    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if not self.distributed:
            return t
        w = self._w
        if self.rank == src:
            w.slots[src] = t
        w.wait()
        if self.rank != src:
            t.copy_(w.slots[src])
        w.wait()
        return t

    def all_gather_async(self, out: torch.Tensor, t: torch.Tensor):
        self.all_gather(out, t)
        return _Done()

    def broadcast_async(self, t: torch.Tensor, src: int):
        """Emulated ranks rendezvous on the host, so the "async" broadcast
        completes before it returns (no overlap to emulate on one stream)."""
        self.broadcast(t, src)
        return _Done()

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if not self.distributed:
            return t
        w = self._w
        w.slots[self.rank] = t
        w.wait()
        acc = w.slots[0].clone()
        for r in range(1, self.world_size):
            v = w.slots[r]
            if op == "sum":
                acc += v
            elif op == "max":
                acc = torch.maximum(acc, v)
            elif op == "min":
                acc = torch.minimum(acc, v)
            else:
                raise ValueError(f"all_reduce op {op!r}")
        w.wait()
        t.copy_(acc)
        return t

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        if not self.distributed:
            out.view(-1).copy_(t.reshape(-1))
            return out
        w = self._w
        w.slots[self.rank] = t.contiguous()
        w.wait()
        n = w.slots[self.rank].numel()
        flat = out.view(-1)
        for r in range(self.world_size):
            flat[r * n:(r + 1) * n].copy_(w.slots[r].reshape(-1))
        w.wait()
        return out

    def barrier(self) -> None:
        if self.distributed:
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            self._w.wait()

    def send(self, t: torch.Tensor, dst: int):
        self._w.box(self.rank, dst).put(t.clone())
        return _Done()

    def recv(self, t: torch.Tensor, src: int):
        return _RecvReq(self._w.box(src, self.rank), t, self._w.timeout_s)

    def sendrecv(self, send_t: torch.Tensor, dst: int, recv_t: torch.Tensor, src: int) -> list:
        return [self.send(send_t, dst), self.recv(recv_t, src)]

    def global_rank(self, r: int) -> int:
        return r

    def subgroup(self, ranks: list[int]) -> Communicator:
        key = tuple(ranks)
        w = self._w
        with w.lock:
            entry = w.subworlds.get(key)
            if entry is None:
                entry = [_World(len(ranks), w.timeout_s), 0]
                w.subworlds[key] = entry
            entry[1] += 1
        # every rank of the parent calls subgroup with the same list (torch
        # semantics); wait for all of them so the registry entry is shared
        w.wait()
        with w.lock:
            if w.subworlds.get(key) is entry and entry[1] == self.world_size:
                del w.subworlds[key]  # next call with the same ranks builds a fresh world
        w.wait()
        if self.rank not in ranks:
            return Communicator(0, 1, self.device, "emulated", None)
        return EmulatedComm(entry[0], ranks.index(self.rank), self.device)


def make_world(size: int, device: str | torch.device = "cpu", timeout_s: float = 300.0) -> list[EmulatedComm]:
    """P communicators sharing one emulated world (hand one to each thread)."""
    if size < 1:
        raise ValueError("world size must be >= 1")
    w = _World(size, timeout_s)
    dev = torch.device(device)
    return [EmulatedComm(w, r, dev) for r in range(size)]


def run_emulated(size: int, fn: Callable[[EmulatedComm], Any], device: str | torch.device = "cpu",
                 timeout_s: float = 300.0) -> list[Any]:
    """Run fn(comm) on `size` emulated ranks (threads); returns the per-rank
    results in rank order, or re-raises the first failing rank's exception."""
    comms = make_world(size, device, timeout_s)
    results: list[Any] = [None] * size
    errors: list[BaseException | None] = [None] * size
    dev = torch.device(device)

    def body(r: int) -> None:
        try:
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            results[r] = fn(comms[r])
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors[r] = e
            comms[r]._w.abort()

    threads = [threading.Thread(target=body, args=(r,), name=f"emu-rank{r}", daemon=True) for r in range(size)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout_s)
    if any(t.is_alive() for t in threads):
        comms[0]._w.abort()
        raise TimeoutError(f"emulated world of {size} ranks did not finish in {timeout_s} s")
    first = next((e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)), None)
    if first is None:
        first = next((e for e in errors if e is not None), None)
    if first is not None:
        raise first
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    return results
