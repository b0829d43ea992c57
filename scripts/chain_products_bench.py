"""Micro-benchmark of DistributedRBT's chain products on one MI355X:
drbt_exec.hip's chain kernels (W = Dk B with D -= L W in one launch; D -= L W
alone) against the same products as dgemm.hip launches, warm (same operands
every launch) and rotating over 64 operand sets (64 x 5 x 128 KB = 40 MB,
beyond the L2s, inside the MALL).  Per-launch time from hipEvents around
200 back-to-back launches.

  python scripts/chain_products_bench.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from gelim import _native  # noqa: E402


def main() -> None:
    lib = _native.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    sets = [[torch.randn(128, 128, dtype=torch.float64, device=dev) for _ in range(5)] for _ in range(64)]

    def fused(o, w):
        Dk, B, W, L, D = o
        lib.gelim_drbt_chain_products(Dk.data_ptr(), B.data_ptr(), W.data_ptr(), L.data_ptr(), D.data_ptr(), w, s)

    def two(o, w):
        Dk, B, W, L, D = o
        if w:
            lib.gelim_gpu_dgemm_ex(W.data_ptr(), 128, Dk.data_ptr(), 128, B.data_ptr(), 128, 128, 128, 128, 1.0, 0, 0, s)
        lib.gelim_gpu_dgemm_ex(D.data_ptr(), 128, L.data_ptr(), 128, W.data_ptr(), 128, 128, 128, 128, -1.0, 1, 0, s)

    for name, fn in (("chain kernel", fused), ("dgemm launches", two)):
        for w in (1, 0):
            for rot in (False, True):
                for _ in range(20):
                    fn(sets[0], w)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(200):
                    fn(sets[i % 64] if rot else sets[0], w)
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 200
                what = "W + D" if w else "D only"
                print(f"{name:15s} {what:7s} {'rotating' if rot else 'warm':8s} {us:7.2f} us per step")


if __name__ == "__main__":
    main()
