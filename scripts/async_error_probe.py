"""Does ncclCommGetAsyncError (gelim_rccl_async_error) block while the
communicator has work queued behind a long kernel, and does it stall a
collective issued meanwhile?  (Diagnostic for the RCCL watchdog.)"""
import os
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29535")
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.parallel import comm as C  # noqa: E402
from gelim.utils.tensors import ptr  # noqa: E402

comm = C.init_from_env(backend="nccl", device="cuda:0", force_pg=True)
dev = comm.device
lib = _native.lib()
t = torch.zeros(4096, dtype=torch.float64, device=dev)
words = torch.zeros(2, dtype=torch.int32, device=dev)
cur = torch.cuda.current_stream(dev)
cs = comm.comm_stream()
nc = comm.rccl()
h = nc.handle
C.watchdog().stop()
comm.broadcast(t, 0)
torch.cuda.synchronize()
log = []
stop = threading.Event()


def poller():
    t0 = time.perf_counter()
    while not stop.is_set():
        a = time.perf_counter()
        rc = lib.gelim_rccl_async_error(h)
        log.append((a - t0, time.perf_counter() - a, rc))
        time.sleep(0.01)


for mode in ("no poller", "poller"):
    th = None
    if mode == "poller":
        stop.clear()
        th = threading.Thread(target=poller)
        th.start()
        time.sleep(0.05)
    words.zero_()
    _native.check(lib.gelim_gpu_probe_kernel(cur.cuda_stream, ptr(words), 0, 100_000_000), "probe")
    time.sleep(0.1)
    cs.wait_stream(cur)
    a = time.perf_counter()
    lib.gelim_rccl_bcast(h, t.data_ptr(), t.numel(), 0, 0, cs.cuda_stream)
    issue = time.perf_counter() - a
    a = time.perf_counter()
    lib.gelim_rccl_allreduce(h, t.data_ptr(), t.data_ptr(), t.numel(), 0, 0, cs.cuda_stream)
    issue2 = time.perf_counter() - a
    torch.cuda.synchronize()
    if th is not None:
        stop.set()
        th.join()
    longest = max((x[1] for x in log), default=0.0)
    print(f"{mode:10s}: bcast issue {issue:.4f} s, allreduce issue {issue2:.4f} s; async_error calls {len(log)}, "
          f"longest {longest:.4f} s, codes {sorted(set(x[2] for x in log))}", flush=True)
C.destroy()
