"""Bisect of the round-4 bench-order slowdown: run the named sections in
order, then time the single-GPU 8192 solve.  Sections: t0 = DistributedGauss
2048 tail=0, te = DistributedGauss 2048 (tail engine), s2 = GaussSolver 2048
graph solve, d8 = DistributedGauss 8192."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import gelim  # noqa: E402
from gelim.parallel import comm as C  # noqa: E402

comm = C.init_from_env(timeout_s=300)
dev = comm.device
for sec in sys.argv[1:]:
    if sec == "t0":
        bench.bench_dist_gauss(comm, gelim, torch, 2048, tail=0)
    elif sec == "te":
        bench.bench_dist_gauss(comm, gelim, torch, 2048)
    elif sec == "s2":
        s = gelim.GaussSolver(2048, backend="hip", device=dev)
        s.solve(gelim.random_system(2048, seed=3, device=dev))
        torch.cuda.synchronize()
        s.close()
    elif sec == "d8":
        bench.bench_dist_gauss(comm, gelim, torch, 8192)
    elif sec == "rbt":
        bench.bench_dist_rbt(comm, gelim, torch, 8192)
    elif sec == "mm":
        bench.bench_matmul(gelim, torch, dev)
    elif sec == "head":
        src = gelim.random_system(2048, seed=1234, device=dev)
        solver = gelim.GaussSolver(2048, backend="hip", device=dev, use_graph=False)
        for _ in range(25):
            solver.solve(src)
        torch.cuda.synchronize()
        solver.close()
    elif sec == "ec":
        torch.cuda.empty_cache()
    elif sec.startswith("streams"):  # streamsN: N torch pool streams, each used once
        for _ in range(int(sec[7:])):
            st = torch.cuda.Stream(dev)
            with torch.cuda.stream(st):
                torch.zeros(1, device=dev).add_(1)
        torch.cuda.synchronize()
    elif sec.startswith("hipstreams"):  # hipstreamsN: N native streams created (and kept) by plans
        keep = [gelim.GaussSolver(64, backend="hip", device=dev) for _ in range(int(sec[10:]))]
        for k in keep:
            k.solve(gelim.random_system(64, seed=1, device=dev))
        torch.cuda.synchronize()
import os  # noqa: E402

q = os.environ.get("GPU_MAX_HW_QUEUES")
if os.environ.get("FINAL") == "t0":  # the dist 2048 panels (tail=0) solve, 4 fresh timings
    ts = [bench.bench_dist_gauss(comm, gelim, torch, 2048, tail=0)["time_s"] * 1e3 for _ in range(4)]
    print(f"Q={q} {' '.join(sys.argv[1:]) or '(none)'} -> dist 2048 tail=0 " + " ".join(f"{t:.2f}" for t in ts)
          + " ms", flush=True)
else:
    t = bench.bench_single(comm, gelim, torch, 8192, seed=77)["time_s"]
    print(f"Q={q} {' '.join(sys.argv[1:]) or '(none)'} -> single 8192 {t * 1e3:.2f} ms", flush=True)
from gelim.utils.tensors import side_stream_stats  # noqa: E402

print(f"   side streams probed / parked: {side_stream_stats()}", flush=True)
