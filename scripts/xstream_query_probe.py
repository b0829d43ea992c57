"""Host time of Event.query() for an event recorded on a stream that waits
(hipStreamWaitEvent) on another stream's running 1 s kernel -- the
completion events the RCCL watchdog polls (diagnostic)."""
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from gelim import _native  # noqa: E402
from gelim.utils.tensors import dedicated_stream, ptr  # noqa: E402

dev = torch.device("cuda:0")
lib = _native.lib()
words = torch.zeros(2, dtype=torch.int32, device=dev)
cur = torch.cuda.current_stream(dev)
cs = dedicated_stream(dev, "comm")
torch.cuda.synchronize()


def case(label, in_thread, query_api):
    words.zero_()
    torch.cuda.synchronize()
    _native.check(lib.gelim_gpu_probe_kernel(cur.cuda_stream, ptr(words), 0, 100_000_000), "probe")
    cs.wait_stream(cur)
    ev = torch.cuda.Event()
    ev.record(cs)
    out = {}

    def q():
        a = time.perf_counter()
        out["v"] = query_api(ev)
        out["dt"] = time.perf_counter() - a

    if in_thread:
        th = threading.Thread(target=q)
        th.start()
        a = time.perf_counter()
        time.sleep(0.001)
        out["main_sleep_1ms"] = time.perf_counter() - a
        th.join()
    else:
        q()
    torch.cuda.synchronize()
    print(f"{label:45s} query {out['dt']:.4f} s -> {out['v']}  main sleep(1ms) took {out.get('main_sleep_1ms', 0):.4f} s",
          flush=True)


def raw_query(ev):
    return lib.gelim_gpu_event_query(ev.cuda_event) if hasattr(lib, "gelim_gpu_event_query") else None


case("torch Event.query, main thread", False, lambda e: e.query())
case("torch Event.query, second thread", True, lambda e: e.query())
