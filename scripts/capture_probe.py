"""Which ways of issuing a torch.distributed (RCCL) collective survive hipGraph
capture with ProcessGroupNCCL's watchdog running?  One variant per process:

  main     sync broadcast on the capture stream itself
  joined   sync broadcast under a dedicated stream that joined the capture
           through an event (parallel/comm.py's _on_comm_stream)
  async    async_op=True broadcast (torch's internal RCCL stream), wait()

Each: warm-up eager, capture 200 broadcasts, sleep 3 s (watchdog polls),
replay 3x, sleep 1 s.  Prints one JSON line.

  python scripts/capture_probe.py VARIANT
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    variant = sys.argv[1]
    import torch
    import torch.distributed as dist

    from gelim.parallel import comm as C
    from gelim.utils.tensors import dedicated_stream

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    comm = C.init_from_env(backend="nccl", force_pg=True)
    dev = comm.device
    t = torch.arange(4096, dtype=torch.float64, device=dev)
    cs = dedicated_stream(dev, "comm")

    def issue():
        if variant == "main":
            dist.broadcast(t, 0)
        elif variant == "joined":
            cur = torch.cuda.current_stream(dev)
            cs.wait_stream(cur)
            with torch.cuda.stream(cs):
                dist.broadcast(t, 0)
                ev = torch.cuda.Event()
                ev.record(cs)
            cur.wait_event(ev)
        else:
            dist.broadcast(t, 0, async_op=True).wait()
        t.add_(1.0)

    issue()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        for _ in range(200):
            issue()
    time.sleep(3)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    time.sleep(1)
    print(json.dumps({"variant": variant, "ok": True, "t0": float(t[0].item())}), flush=True)
    C.destroy()


if __name__ == "__main__":
    main()
