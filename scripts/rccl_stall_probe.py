"""Host time of each step of a native one-rank RCCL collective issued while
the current stream runs a 1 s kernel (diagnostic for the RCCL watchdog):
does anything in the issue path block the host until the stream drains?"""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.parallel import comm as C  # noqa: E402
from gelim.utils.tensors import ptr  # noqa: E402

comm = C.init_from_env(backend="nccl", device="cuda:0", force_pg=True)
dev = comm.device
lib = _native.lib()
t = torch.zeros(4096, dtype=torch.float64, device=dev)
words = torch.zeros(2, dtype=torch.int32, device=dev)
nc = comm.rccl()
cs = comm.comm_stream()
cur = torch.cuda.current_stream(dev)
comm.broadcast(t, 0)
torch.cuda.synchronize()


def spin():
    words.zero_()
    _native.check(lib.gelim_gpu_probe_kernel(cur.cuda_stream, ptr(words), 0, 100_000_000), "probe")


def step(label, fn):
    a = time.perf_counter()
    fn()
    print(f"  {label:40s} {time.perf_counter() - a:.4f} s", flush=True)


for name, op in (("bcast", lambda s: nc.bcast(t, 0, s)), ("allreduce", lambda s: nc.allreduce(t, "sum", s)),
                 ("allgather", lambda s: nc.allgather(t.clone(), t, s)),
                 ("sendrecv", lambda s: nc.sendrecv(t, 0, t.clone(), 0, s))):
    print(name, "on the comm stream behind a 1 s kernel:", flush=True)
    spin()
    step("cs.wait_stream(cur)", lambda: cs.wait_stream(cur))
    step("collective on cs", lambda: op(cs.cuda_stream))
    ev = torch.cuda.Event()
    step("event record", lambda: ev.record(cs))
    step("query", lambda: ev.query())
    step("synchronize", torch.cuda.synchronize)
    print(name, "on the current stream behind a 1 s kernel:", flush=True)
    spin()
    step("collective on cur", lambda: op(cur.cuda_stream))
    step("synchronize", torch.cuda.synchronize)
C.destroy()
