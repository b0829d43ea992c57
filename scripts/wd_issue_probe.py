"""Step timing of Communicator.broadcast_async behind a 2 s kernel, with and
without the RCCL watchdog thread (diagnostic)."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.update(RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29536")
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
comm.broadcast(t, 0)
comm.synchronize()
nc = comm.rccl()


def run(label):
    words.zero_()
    _native.check(lib.gelim_gpu_probe_kernel(cur.cuda_stream, ptr(words), 0, 100_000_000), "probe")
    st = []
    a = time.perf_counter()
    cs.wait_stream(cur)
    st.append(("wait_stream", time.perf_counter() - a))
    with torch.cuda.stream(cs):
        st.append(("enter", time.perf_counter() - a))
        nc.bcast(t, 0, cs.cuda_stream)
        st.append(("bcast", time.perf_counter() - a))
        ev = torch.cuda.Event()
        ev.record(cs)
        st.append(("record", time.perf_counter() - a))
    t.record_stream(cs)
    st.append(("record_stream", time.perf_counter() - a))
    h = C._Event(ev)
    st.append(("_Event", time.perf_counter() - a))
    h.wait()
    st.append(("wait", time.perf_counter() - a))
    print(label, " ".join(f"{k}={v:.4f}" for k, v in st), flush=True)
    torch.cuda.synchronize()


run("watchdog (120 s):")
C.start_watchdog(timeout_s=0.5, poll_s=0.02)
try:
    run("watchdog (0.5 s):")
except C.CommFailure as e:
    print("raised", e)
wd = C.watchdog()
wd.stop()
C._WATCHDOG.clear()
time.sleep(0.1)
try:
    run("no watchdog thread:")
except C.CommFailure as e:
    print("raised", e)
C.destroy(abort=True)
