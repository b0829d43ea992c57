"""Bench section order check: the single-GPU 8192 solve timed after each of
bench.py's preceding sections, in bench.py's order (round 4: it read 49 ms
inside bench.py vs 34 ms alone)."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import gelim  # noqa: E402
from gelim.parallel import comm as C  # noqa: E402

comm = C.init_from_env(timeout_s=300)
dev = comm.device


def single(tag):
    print(f"single 8192 {tag}: {bench.bench_single(comm, gelim, torch, 8192, seed=77)['time_s'] * 1e3:.2f} ms",
          flush=True)


src = gelim.random_system(2048, seed=1234, device=dev)
solver = gelim.GaussSolver(2048, backend="hip", pivot="partial", device=dev, use_graph=False)
for _ in range(25):
    x = solver.solve(src)
torch.cuda.synchronize()
solver.close()
single("after headline")
bench.bench_matmul(gelim, torch, dev)
single("after matmul_2048")
bench.bench_dist_gauss(comm, gelim, torch, 8192)
single("after dist 8192")
bench.bench_dist_rbt(comm, gelim, torch, 8192)
single("after dist rbt")
bench.bench_dist_gauss(comm, gelim, torch, 2048, tail=0)
bench.bench_dist_gauss(comm, gelim, torch, 2048)
single("after dist 2048 x2")
bench.bench_dist_matmul(comm, gelim, torch, 16384)
single("after dist matmul")
