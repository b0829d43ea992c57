"""Event completion after a cross-stream wait (diagnostic for the RCCL
watchdog): a 1 s kernel on the current stream, then
  A: event recorded on the current stream                      -> must be pending
  B: comm stream waits on current, marker event on comm stream;
     current waits on that event; event recorded on current    -> must be pending
  C: as B but with a native one-rank RCCL broadcast on the comm stream."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29534")
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.parallel import comm as C  # noqa: E402
from gelim.utils.tensors import ptr  # noqa: E402

comm = C.init_from_env(backend="nccl", device="cuda:0", force_pg=True)
dev = comm.device
lib = _native.lib()
t = torch.zeros(4096, dtype=torch.float64, device=dev)
words = torch.zeros(2, dtype=torch.int32, device=dev)
cs = comm.comm_stream()
cur = torch.cuda.current_stream(dev)
comm.broadcast(t, 0)
torch.cuda.synchronize()


def spin():
    words.zero_()
    _native.check(lib.gelim_gpu_probe_kernel(cur.cuda_stream, ptr(words), 0, 100_000_000), "probe")


def pending_after(label, fn):
    spin()
    fn()
    ev = torch.cuda.Event()
    ev.record(cur)
    a = time.perf_counter()
    q = ev.query()
    ev.synchronize()
    print(f"{label:60s} pending={not q}  drained after {time.perf_counter() - a:.3f} s", flush=True)
    torch.cuda.synchronize()


pending_after("A: nothing", lambda: None)


def b():
    cs.wait_stream(cur)
    e = torch.cuda.Event()
    e.record(cs)
    cur.wait_event(e)


pending_after("B: cs waits cur, marker on cs, cur waits marker", b)


def c():
    h = comm.broadcast_async(t, 0)
    h.wait()


pending_after("C: broadcast_async + wait (native RCCL)", c)


def d():
    cs.wait_stream(cur)
    e = torch.cuda.Event()
    e.record(cs)


pending_after("D: cs waits cur, marker on cs (cur does not wait)", d)


def e_():
    with torch.cuda.stream(cs):
        lib.gelim_rccl_bcast(comm.rccl().handle, t.data_ptr(), t.numel(), 0, 0, cs.cuda_stream)


pending_after("E: bare RCCL bcast on cs (no waits)", e_)
C.destroy()
