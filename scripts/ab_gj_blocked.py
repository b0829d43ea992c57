"""A/B of the diagonal-block inverse forms (GELIM_GJ_BLOCKED=0: one barrier
per pivot; 1 / 2: 32- / 16-pivot blocks with MFMA updates): the kernel alone, and the
hip-rbt solves at 2048 and 8192 (time, corrections, backward error).

  python scripts/ab_gj_blocked.py
"""
import os
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

dev = torch.device("cuda:0")
lib = gelim._native.lib()
sh = stream_handle(dev)
Af = torch.randn(128, 130, dtype=torch.float64, device=dev)
Af[:, :128] += 16 * torch.eye(128, dtype=torch.float64, device=dev)
A = Af[:, :128]  # a strided block, leading dimension 130
D = torch.empty(128, 128, dtype=torch.float64, device=dev)
info = torch.full((1,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
for form in ("0", "1", "2"):
    os.environ["GELIM_GJ_BLOCKED"] = form
    for _ in range(3):
        lib.gelim_rbt_block_inverse(ptr(A), 130, 0, ptr(D), ptr(info), sh)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        lib.gelim_rbt_block_inverse(ptr(A), 130, 0, ptr(D), ptr(info), sh)
    e1.record()
    torch.cuda.synchronize()
    ref = torch.linalg.inv(A)
    print(f"GELIM_GJ_BLOCKED={form}: inverse {e0.elapsed_time(e1) * 10:.1f} us, "
          f"max rel diff vs torch {((D - ref).abs().max() / ref.abs().max()).item():.2e}", flush=True)
for n in (2048, 8192):
    aug = gelim.random_system(n, seed=31 + n, device=dev)
    for form in ("0", "1", "2"):
        os.environ["GELIM_GJ_BLOCKED"] = form
        s = gelim.GaussSolver(n, backend="hip-rbt", device=dev)
        s.solve(aug)
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            x = s.solve(aug)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"n={n} GELIM_GJ_BLOCKED={form}: hip-rbt {statistics.median(ts) * 1e3:.3f} ms (min "
              f"{min(ts) * 1e3:.3f}), corrections {s.last_steps}, fallback {s.last_fallback}, "
              f"error {gelim.ops.gauss.error_metric(x):.2e}", flush=True)
        s.close()
