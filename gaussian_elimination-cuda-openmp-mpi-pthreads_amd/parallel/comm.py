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

import ctypes
import datetime
import os
import threading
import time
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

    def __init__(self, ev: torch.cuda.Event, what: str = "collective"):
        self.ev = ev
        _watch(ev, what)

    def wait(self) -> bool:
        torch.cuda.current_stream().wait_event(self.ev)
        return True

    def is_completed(self) -> bool:
        return self.ev.query()


class CommFailure(RuntimeError):
    """A device collective did not complete: a peer died or hung (no
    progress within the watchdog's timeout), or RCCL reported an
    asynchronous communicator error.  Every native communicator of the
    process has been aborted (ncclCommAbort) when this is raised; the
    process cannot issue further collectives and should exit."""


class CommWatchdog:
    """Failure detection for libgelim's native RCCL collectives (SURVEY §5.3:
    async-error polling + a watchdog timeout).  The reference's MPI program
    has none -- MPI_ERRORS_ARE_FATAL, no handler
    (OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:289-297) -- and a dead
    peer there ends the job; here a dead or stuck peer must not leave the
    surviving ranks blocked forever in a device wait.

    One daemon thread per process (started with the first native
    communicator).  Every `poll_s` it
      * asks each live communicator for its asynchronous error
        (ncclCommGetAsyncError through gelim_rccl_async_error);
      * queries the completion events of the outstanding collectives
        (recorded after every native collective issued outside a hipGraph
        capture) and fails when the oldest is older than `timeout_s`.
    Failing = ncclCommAbort on every native communicator (RCCL kernels in
    flight poll the abort flag and exit, so a blocked device wait returns),
    then the error is raised on the main thread: directly by the solvers'
    wait points (`Communicator.synchronize` / `Communicator.item`, event-query
    loops with the same deadline), otherwise asynchronously
    (PyThreadState_SetAsyncExc) once the main thread runs Python again.
    The thread pauses while a hipGraph is being captured (`paused()`):
    nothing it could query exists yet, and queries during a capture are
    not safe."""

    def __init__(self, timeout_s: float, poll_s: float = 0.05):
        self.timeout_s = float(timeout_s)
        self.poll_s = poll_s
        self.error: CommFailure | None = None
        self._raised = False
        self._pending: list[tuple[float, torch.cuda.Event, str]] = []
        self._lock = threading.Lock()
        self._pause = 0
        self._in_wait = 0
        self._stop = threading.Event()
        self._main = threading.main_thread().ident
        self._thread = threading.Thread(target=self._run, name="gelim-rccl-watchdog", daemon=True)
        self._thread.start()

    # -- bookkeeping ----------------------------------------------------------
    def track(self, ev: torch.cuda.Event, what: str) -> None:
        with self._lock:
            self._pending.append((time.monotonic(), ev, what))

    def paused(self):
        wd = self

        class _P:
            def __enter__(self):
                with wd._lock:
                    wd._pause += 1

            def __exit__(self, *exc):
                with wd._lock:
                    wd._pause -= 1
                    # ages restart: a capture's own host time is not a stall
                    now = time.monotonic()
                    wd._pending = [(now, e, w) for _, e, w in wd._pending]
                return False

        return _P()

    def check(self) -> None:
        """Raise the recorded failure (once per failure on the main path)."""
        if self.error is not None:
            self._raised = True
            raise self.error

    def fail(self, msg: str) -> None:
        """Record the failure; the watchdog thread aborts the communicators
        (ncclCommAbort can wait for the device to drain, so the raise on the
        main thread never waits for it: from here on every native call
        raises the recorded error instead of touching a communicator)."""
        with self._lock:
            if self.error is not None:
                return
            self.error = CommFailure(msg)
            self._pending.clear()

    def _abort_all(self) -> None:
        for nc in list(_NATIVE):
            try:
                nc.destroy(abort=True)
            except Exception:  # noqa: BLE001 - aborting is best effort
                pass

    def wait_event(self, ev: torch.cuda.Event, what: str) -> None:
        """Host wait for ev as an event-query loop: raises CommFailure when
        the watchdog failed, or when ev is not complete after timeout_s."""
        t0 = time.monotonic()
        spins = 0
        with self._lock:
            self._in_wait += 1
        try:
            while not ev.query():
                self.check()
                if time.monotonic() - t0 > self.timeout_s:
                    self.fail(f"{what}: device work (collectives included) not finished after "
                              f"{self.timeout_s:.1f} s -- a peer rank died or hung")
                    self.check()
                spins += 1
                if spins > 2000:  # ~2 ms of spinning, then yield the CPU
                    time.sleep(1e-4)
            self.check()
        finally:
            with self._lock:
                self._in_wait -= 1

    def stop(self) -> None:
        self._stop.set()

    # -- the thread -----------------------------------------------------------
    def _run(self) -> None:
        aborted = False
        while not self._stop.wait(self.poll_s):
            if self.error is not None:
                self._deliver()  # first: the raise does not wait for the abort
                if not aborted:
                    aborted = True
                    self._abort_all()
                continue
            with self._lock:
                if self._pause:
                    continue
                pending = list(self._pending)
            try:
                for nc in list(_NATIVE):
                    rc = nc.async_error()
                    if rc:
                        self.fail(f"RCCL asynchronous error on communicator {nc.key!r}: {rc}")
                        break
                if self.error is None and pending:
                    now = time.monotonic()
                    done = set()
                    for t, ev, what in pending:
                        if ev.query():
                            done.add(id(ev))
                        elif now - t > self.timeout_s:
                            self.fail(f"{what}: not complete after {now - t:.1f} s (timeout {self.timeout_s:.1f} "
                                      "s) -- a peer rank died or hung")
                            break
                    with self._lock:
                        self._pending = [p for p in self._pending if id(p[1]) not in done]
            except Exception as e:  # noqa: BLE001 - a failing query is itself a failure
                if self.error is None:
                    self.fail(f"watchdog query failed: {e!r}")

    def _deliver(self) -> None:
        """Raise the failure in the main thread if no wait point did."""
        with self._lock:
            if self._raised or self._in_wait or self._main is None:
                return
            self._raised = True
        ctypes.pythonapi.PyThreadState_SetAsyncExc(ctypes.c_ulong(self._main), ctypes.py_object(CommFailure))


_WATCHDOG: list[CommWatchdog] = []  # the process's watchdog (at most one)
_WATCHDOG_TIMEOUT = [600.0]         # init_from_env's timeout_s


def watchdog() -> CommWatchdog | None:
    return _WATCHDOG[0] if _WATCHDOG else None


def start_watchdog(timeout_s: float | None = None, poll_s: float = 0.05) -> CommWatchdog:
    """The process's watchdog (created on first use; timeout_s defaults to
    init_from_env's)."""
    if not _WATCHDOG:
        _WATCHDOG.append(CommWatchdog(_WATCHDOG_TIMEOUT[0] if timeout_s is None else timeout_s, poll_s))
    elif timeout_s is not None:
        _WATCHDOG[0].timeout_s = float(timeout_s)
    return _WATCHDOG[0]


def _tracking() -> CommWatchdog | None:
    """The watchdog if collectives are to be tracked now: not while a capture
    is in progress (Communicator.capturing): the event would be a graph node,
    and a graph's replay is waited for by the wait points.  (The pause flag,
    not a runtime capture query per collective: the only Python-level
    capture of collectives is DistributedRBT._replay, which sets it.)"""
    wd = watchdog()
    return wd if wd is not None and not wd._pause else None


def _watch(ev: torch.cuda.Event, what: str) -> None:
    """Track a native collective's completion event."""
    wd = _tracking()
    if wd is not None:
        wd.track(ev, what)


_DTYPE = {torch.float64: 0, torch.float32: 1, torch.int32: 2, torch.int64: 3, torch.uint8: 4}
_OP = {"sum": 0, "max": 1, "min": 2}
_NATIVE: list = []  # every live NativeRccl of the process (destroy() releases them)
_NATIVE_LOCK = threading.RLock()  # destroy vs the watchdog's async-error queries


class NativeRccl:
    """One RCCL communicator owned by libgelim (csrc/comm/rccl_comm.hip):
    each collective is one RCCL call on a caller-chosen stream, ~3 us of host
    time against ~65 us through ProcessGroupNCCL, capturable into hipGraphs
    (torch's watchdog queries the events of collectives recorded during a
    capture and aborts the process).  The RCCL is torch's own librccl.so (one
    instance in the process); the 128-byte unique id of the communicator goes
    from its rank 0 to the others through the process group's store, under
    `key`.  Creation is collective over the nranks members."""

    def __init__(self, key: str, nranks: int, rank: int, device: torch.device):
        import ctypes

        from .. import _native

        self.lib = lib = _native.lib()
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        _native.check(lib.gelim_rccl_load(path.encode()), "rccl_load")
        store = dist.distributed_c10d._get_default_store()
        idb = (ctypes.c_uint8 * 128)()
        if rank == 0:
            _native.check(lib.gelim_rccl_unique_id(idb), "rccl_unique_id")
            store.set(key, bytes(idb))
        else:
            ctypes.memmove(idb, store.get(key), 128)
        h = ctypes.c_void_p()
        with torch.cuda.device(device):
            _native.check(lib.gelim_rccl_comm_create(ctypes.byref(h), idb, nranks, rank), "rccl_comm_create")
        self.handle, self.nranks, self.rank, self.device = h.value, nranks, rank, device
        self.key = key
        _NATIVE.append(self)
        start_watchdog()

    def check(self, rc: int, what: str) -> None:
        from .. import _native

        _native.check(rc, what)
        wd = _tracking()
        if wd is not None:
            # synchronous collectives: their completion is tracked like the
            # asynchronous ones' (an event on the stream they were issued on)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            wd.track(ev, what)

    def _h(self):
        """The live handle; after a failure (abort pending or done), the
        failure that caused it."""
        wd = watchdog()
        if wd is not None and wd.error is not None:
            raise wd.error
        if not self.handle:
            raise CommFailure(f"RCCL communicator {self.key!r} was destroyed")
        return self.handle

    def async_error(self) -> int:
        with _NATIVE_LOCK:  # never on a communicator being destroyed
            h = self.handle
            return self.lib.gelim_rccl_async_error(h) if h else 0

    @staticmethod
    def dtype(t: torch.Tensor) -> int:
        try:
            return _DTYPE[t.dtype]
        except KeyError:
            raise TypeError(f"RCCL collective on {t.dtype}") from None

    def bcast(self, t: torch.Tensor, root: int, stream: int) -> None:
        self.check(self.lib.gelim_rccl_bcast(self._h(), t.data_ptr(), t.numel(), self.dtype(t), root, stream),
                   "rccl_bcast")

    def allreduce(self, t: torch.Tensor, op: str, stream: int) -> None:
        self.check(self.lib.gelim_rccl_allreduce(self._h(), t.data_ptr(), t.data_ptr(), t.numel(), self.dtype(t),
                                                 _OP[op], stream), "rccl_allreduce")

    def allgather(self, out: torch.Tensor, t: torch.Tensor, stream: int) -> None:
        self.check(self.lib.gelim_rccl_allgather(self._h(), t.data_ptr(), out.data_ptr(), t.numel(),
                                                 self.dtype(t), stream), "rccl_allgather")

    def sendrecv(self, send_t: torch.Tensor | None, dst: int, recv_t: torch.Tensor | None, src: int,
                 stream: int) -> None:
        ref = send_t if send_t is not None else recv_t
        self.check(self.lib.gelim_rccl_sendrecv(
            self._h(), send_t.data_ptr() if send_t is not None else None,
            send_t.numel() if send_t is not None else 0, dst,
            recv_t.data_ptr() if recv_t is not None else None, recv_t.numel() if recv_t is not None else 0, src,
            self.dtype(ref), stream), "rccl_sendrecv")

    def destroy(self, abort: bool = False) -> None:
        with _NATIVE_LOCK:
            h, self.handle = self.handle, None
            if h:
                self.lib.gelim_rccl_comm_destroy(h, int(abort))
        if self in _NATIVE:
            _NATIVE.remove(self)


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
    key: str = "world"  # store key prefix of this communicator's native RCCL id
    _rccl: object = field(default=None, repr=False, compare=False)
    _rccl_aux: object = field(default=None, repr=False, compare=False)

    # -- collectives ------------------------------------------------------
    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.pg

    @property
    def native(self) -> bool:
        """RCCL ranks run their device collectives through libgelim's own
        RCCL communicator (NativeRccl) on chosen streams; GELIM_COMM=torch
        routes them through torch.distributed instead (A/B, and the
        fallback if a native communicator cannot be created)."""
        return (self.backend == "nccl" and self.device.type == "cuda" and self.distributed
                and os.environ.get("GELIM_COMM", "native") != "torch")

    def rccl(self) -> NativeRccl:
        if self._rccl is None:
            self._rccl = NativeRccl(f"gelim_rccl/{self.key}", self.world_size, self.rank, self.device)
        return self._rccl

    def rccl_aux(self, name: str) -> NativeRccl:
        """A further native communicator over the same ranks (collective:
        every rank asks for the same names in the same order).  Two
        communicators progress independently, so a collective on one never
        waits behind a long one on the other (DistributedRBT: the chain's
        small messages beside the bulk columns)."""
        if self._rccl_aux is None:
            self._rccl_aux = {}
        if name not in self._rccl_aux:
            self._rccl_aux[name] = NativeRccl(f"gelim_rccl/{self.key}/{name}", self.world_size, self.rank,
                                              self.device)
        return self._rccl_aux[name]

    def comm_stream(self) -> torch.cuda.Stream:
        """The stream this rank's asynchronous collectives run on: a
        process-lifetime stream on a hardware queue of its own, probed to run
        beside the default stream and the lookahead side stream
        (utils/tensors.dedicated_stream) -- not torch's internal RCCL
        stream, a pool stream whose hardware queue nobody checks: HIP maps
        streams onto GPU_MAX_HW_QUEUES (4) queues, and a collective on the
        side stream's queue would wait behind the whole trailing update
        (profiles/hw_queues_r4.txt).  (Through torch, a synchronous
        collective runs on the CURRENT stream in torch >= 2.7, so it is
        issued under this stream.)"""
        if self._cstream is None:
            from ..utils.tensors import dedicated_stream

            self._cstream = dedicated_stream(self.device, "comm")
        return self._cstream

    def _on_comm_stream(self, issue, *tensors: torch.Tensor) -> _Event:
        cs = self.comm_stream()
        cs.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(cs):
            issue(cs.cuda_stream)
            ev = torch.cuda.Event()
            ev.record(cs)
        for t in tensors:  # the caching allocator must not hand these out before cs is done
            t.record_stream(cs)
        return _Event(ev)

    def _cur(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    @property
    def staged(self) -> bool:
        """gloo ranks holding device tensors (several ranks sharing one GPU,
        which RCCL refuses): broadcast and all_reduce use gloo's own device
        path (asynchronous, stream-ordered); all_gather and point-to-point
        ops, which it lacks for device tensors, go through host memory."""
        return self.backend == "gloo" and self.device.type == "cuda"

    def broadcast(self, t: torch.Tensor, src: int) -> torch.Tensor:
        if self.native:
            self.rccl().bcast(t, src, self._cur())
        elif self.distributed:
            dist.broadcast(t, src=self.global_rank(src), group=self.group)
        return t

    def broadcast_async(self, t: torch.Tensor, src: int):
        """Non-blocking broadcast: returns a handle whose wait() makes the
        current stream wait for the data (the collective runs on the
        communicator's stream, after the work already queued on the current
        one)."""
        if self.native:
            nc = self.rccl()
            return self._on_comm_stream(lambda s: nc.bcast(t, src, s), t)
        if self.distributed and self.backend == "nccl" and self.device.type == "cuda":
            return self._on_comm_stream(lambda s: dist.broadcast(t, src=self.global_rank(src), group=self.group))
        if self.distributed:
            return dist.broadcast(t, src=self.global_rank(src), group=self.group, async_op=True)
        return _Done()

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self.native:
            self.rccl().allreduce(t, op, self._cur())
        elif self.distributed:
            rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
            dist.all_reduce(t, op=rop, group=self.group)
        return t

    def all_gather(self, out: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
        """out: (world_size * t.numel()) contiguous tensor."""
        if self.native:
            self.rccl().allgather(out, t.contiguous(), self._cur())
        elif self.distributed and self.staged:
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
        src = t.contiguous().view(-1)
        if self.native:
            nc = self.rccl()
            return self._on_comm_stream(lambda s: nc.allgather(out, src, s), out, src)
        if self.distributed and self.backend == "nccl" and self.device.type == "cuda":
            return self._on_comm_stream(lambda s: dist.all_gather_into_tensor(out.view(-1), src, group=self.group))
        if self.distributed:
            return dist.all_gather_into_tensor(out.view(-1), src, group=self.group, async_op=True)
        out.view(-1).copy_(t.reshape(-1))
        return _Done()

    def barrier(self) -> None:
        if self.distributed:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[self.device.index])
            else:
                dist.barrier(group=self.group)

    def send(self, t: torch.Tensor, dst: int):
        if self.native:  # stream-ordered on the current stream
            self.rccl().sendrecv(t, dst, None, 0, self._cur())
            return _Done()
        if self.staged:
            h = t.detach().cpu()
            return _Staged(dist.isend(h, dst=self.global_rank(dst), group=self.group), h)
        return dist.isend(t, dst=self.global_rank(dst), group=self.group)

    def recv(self, t: torch.Tensor, src: int):
        if self.native:
            self.rccl().sendrecv(None, 0, t, src, self._cur())
            return _Done()
        if self.staged:
            h = torch.empty(t.shape, dtype=t.dtype)
            return _Staged(dist.irecv(h, src=self.global_rank(src), group=self.group), h, t)
        return dist.irecv(t, src=self.global_rank(src), group=self.group)

    def sendrecv(self, send_t: torch.Tensor, dst: int, recv_t: torch.Tensor, src: int) -> list:
        """Send to dst and receive from src as ONE batched p2p operation
        (batch_isend_irecv: RCCL group semantics, so a ring of such calls
        cannot deadlock on serialised send kernels).  Returns the requests."""
        if self.native:
            # one grouped RCCL send/recv on the communicator stream (after the
            # work queued so far on the current one), so a ring step's
            # transfer overlaps the compute queued behind it; wait() makes the
            # current stream wait for it
            nc = self.rccl()
            return [self._on_comm_stream(lambda s: nc.sendrecv(send_t, dst, recv_t, src, s), send_t, recv_t)]
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

    # -- host waits (the wait points of the distributed solvers) ---------------
    def synchronize(self) -> None:
        """Host wait for the work queued on the current stream.  On the
        native RCCL path this is an event-query loop under the watchdog
        (CommWatchdog.wait_event): a collective that a dead or stuck peer
        never completes raises CommFailure after the timeout instead of
        blocking forever in hipDeviceSynchronize."""
        if self.device.type != "cuda":
            return
        wd = watchdog() if self.native else None
        if wd is None:
            torch.cuda.synchronize(self.device)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        wd.wait_event(ev, f"rank {self.rank}: host wait")

    def item(self, t: torch.Tensor):
        """t.item() behind synchronize() (a guarded wait point)."""
        if t.device.type == "cuda" and self.native:
            self.synchronize()
        return t.item()

    def capturing(self):
        """Context for a hipGraph capture of this rank's collectives: the
        watchdog pauses (its event queries are not safe during a capture)."""
        wd = watchdog()
        if wd is None:
            import contextlib

            return contextlib.nullcontext()
        return wd.paused()

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
        self._nsub = getattr(self, "_nsub", 0) + 1  # every rank makes the same calls: same keys
        if self.rank not in ranks:
            return Communicator(0, 1, self.device, self.backend, None)
        key = f"{self.key}/sub{self._nsub}:" + "-".join(map(str, ranks))
        return Communicator(ranks.index(self.rank), len(ranks), self.device, self.backend, g,
                            pg=self.pg, _cstream=self._cstream, key=key)

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
    _WATCHDOG_TIMEOUT[0] = float(timeout_s)
    if _WATCHDOG:
        _WATCHDOG[0].timeout_s = float(timeout_s)
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
    # blocked forever.  ProcessGroupNCCL's async error handling turns a
    # collective that exceeds `timeout_s` (or a communicator error) into an
    # abort on every surviving rank; gloo raises on the same timeout; the
    # solvers' own RCCL communicators are covered by CommWatchdog (same
    # timeout: ncclCommGetAsyncError polling, completion-event ages, guarded
    # host waits, ncclCommAbort + CommFailure).
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return Communicator(rank, world, dev, backend)


def destroy(abort: bool = False) -> None:
    """Release the native RCCL communicators (abort=True: ncclCommAbort,
    after a failed peer -- also what happens when the watchdog has failed)
    and the process group."""
    wd = watchdog()
    if wd is not None:
        abort = abort or wd.error is not None
        wd.stop()
        _WATCHDOG.clear()
    for nc in list(_NATIVE):
        nc.destroy(abort)
    if dist.is_initialized():
        if abort:
            try:
                dist.distributed_c10d._abort_process_group()  # type: ignore[attr-defined]
                return
            except Exception:  # noqa: BLE001 - older torch: plain destroy
                pass
        dist.destroy_process_group()
