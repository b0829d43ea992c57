"""How long does torch.cuda.Event.query() take while the stream it was
recorded on runs a long kernel (main thread, second thread; default stream
and a side stream)?  Diagnostic for the RCCL watchdog's event polling."""
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402
from gelim import _native  # noqa: E402
from gelim.utils.tensors import dedicated_stream, ptr  # noqa: E402

dev = torch.device("cuda:0")
lib = _native.lib()
words = torch.zeros(2, dtype=torch.int32, device=dev)
torch.cuda.synchronize()


def run(stream, label, in_thread):
    words.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        _native.check(lib.gelim_gpu_probe_kernel(stream.cuda_stream, ptr(words), 0, 100_000_000), "probe")
        ev = torch.cuda.Event()
        ev.record(stream)
    t0 = time.perf_counter()
    qs = []

    def body():
        while True:
            a = time.perf_counter()
            d = ev.query()
            qs.append((a - t0, time.perf_counter() - a, d))
            if d:
                break
            time.sleep(0.01)

    if in_thread:
        th = threading.Thread(target=body)
        th.start()
        th.join()
    else:
        body()
    longest = max(q[1] for q in qs)
    print(f"{label:28s} queries={len(qs)} first_query_s={qs[0][1]:.4f} longest_query_s={longest:.4f} "
          f"done_at_s={qs[-1][0]:.3f}", flush=True)


cur = torch.cuda.current_stream(dev)
side = dedicated_stream(dev, "comm")
for s, name in ((cur, "default"), (side, "dedicated")):
    for th in (False, True):
        run(s, f"{name} {'thread' if th else 'main'}", th)
