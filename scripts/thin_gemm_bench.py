"""Thin fp64 GEMM shapes of the randomised block-LDU engine (lu_mixed.hip
factor_la2 at n = 8192, parallel/dist_rbt.py): dgemm.hip's LDS-tiled kernel
(gelim_gpu_dgemm_ex) vs the register-direct thin kernel (dgemm_thin.hip,
variants 1..5), microseconds per call (CUDA events, 50 calls) and TFLOP/s,
each result checked against torch (hipBLAS) fp64.  The event timing of
back-to-back ctypes launches is host-bound below ~10 us; kernel times come
from rocprofv3 (scripts/thin_gemm_prof.sh).

  python scripts/thin_gemm_bench.py [--shape i] > profiles/dgemm_thin_r4.txt
"""
import os
import sys
from pathlib import Path



import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402

SHAPES = [  # M, N, K, accumulate, what
    (128, 8064, 128, 0, "W = D_k A[k, k+1:]"),
    (8064, 128, 128, 1, "block column k+1 -= A[k+1:, k] W"),
    (128, 7936, 128, 1, "block row k+1 -= A[k+1, k] W"),
    (7936, 256, 256, 1, "next pair's panel columns (K = 256)"),
    (256, 7680, 256, 1, "next pair's panel rows (K = 256)"),
    (4096, 128, 128, 1, "mid-factor column update"),
    (128, 4096, 128, 0, "mid-factor W"),
    (1024, 128, 128, 1, "late column update"),
    (8192, 224, 32, 1, "wide-panel leaf update (biglu)"),
]


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, default=-1, help="index into SHAPES (default: all)")
    args = ap.parse_args()
    shapes = SHAPES if args.shape < 0 else [SHAPES[args.shape]]
    dev = torch.device("cuda:0")
    lib = gelim._native.lib()
    sh = stream_handle(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    print(f"{'shape':>22} {'kernel':>10} {'us':>8} {'TF/s':>7} {'rel_err':>9}  what")
    for M, N, K, acc, what in shapes:
        A = torch.randn(M, K + 2, dtype=torch.float64, device=dev, generator=g)[:, :K]
        B = torch.randn(K, N + 2, dtype=torch.float64, device=dev, generator=g)[:, :N]
        C0 = torch.randn(M, N + 2, dtype=torch.float64, device=dev, generator=g)[:, :N]
        ref = (C0 if acc else 0) - A @ B
        flops = 2.0 * M * N * K
        for name, v in [("lds", -1), ("thin1", 1), ("thin2", 2), ("thin3", 3), ("thin4", 4), ("thin5", 5),
                        ("deep6", 6), ("deep7", 7), ("deep8", 8)]:
            C = C0.clone() if True else None
            Cv = torch.empty(M, N + 2, dtype=torch.float64, device=dev)[:, :N]
            Cv.copy_(C0)

            def call():
                if v < 0:
                    return lib.gelim_gpu_dgemm_ex(ptr(Cv), Cv.stride(0), ptr(A), A.stride(0), ptr(B), B.stride(0),
                                                  M, N, K, -1.0, acc, 0, sh)
                return lib.gelim_gpu_dgemm_thin(ptr(Cv), Cv.stride(0), ptr(A), A.stride(0), ptr(B), B.stride(0),
                                                M, N, K, -1.0, acc, v, sh)

            rc = call()
            if rc != 0:
                print(f"{M:>6}x{N:>6}x{K:>4} {name:>10}  skipped (rc {rc})")
                continue
            torch.cuda.synchronize()
            err = ((Cv - ref).abs().max() / ref.abs().max()).item()
            for _ in range(5):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 50
            e0.record()
            for _ in range(reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            print(f"{M:>6}x{N:>6}x{K:>4} {name:>10} {us:8.2f} {flops / us * 1e-6:7.2f} {err:9.1e}  {what}")
            del C


if __name__ == "__main__":
    main()
