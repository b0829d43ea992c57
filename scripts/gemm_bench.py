"""Standalone GEMM timings on one GPU (hipEvent, median of reps): the fp64
MFMA dgemm (dgemm.hip) at the wide-panel engine's trailing-update shapes and
the fp32 MFMA GEMM (gemm_f32.hip) at square sizes.

  python scripts/gemm_bench.py [f64|f32|all]
"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import gelim  # noqa: E402
from gelim import _native  # noqa: E402
from gelim.utils.tensors import ptr, stream_handle  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3)
    return sorted(ts)[len(ts) // 2]


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    dev = torch.device("cuda:0")
    lib = _native.lib()
    sh = stream_handle(dev)
    if what in ("f64", "all"):
        for M, N, K in [(8192, 8192, 256), (6144, 6144, 256), (4096, 4096, 256), (2048, 2048, 256),
                        (8192, 224, 32), (8192, 256, 256), (4096, 4096, 4096)]:
            ld = N + 2
            C = torch.randn(M, ld, dtype=torch.float64, device=dev)
            A = torch.randn(M, K, dtype=torch.float64, device=dev)
            B = torch.randn(K, ld, dtype=torch.float64, device=dev)
            dt = timeit(lambda: _native.check(lib.gelim_gpu_dgemm(ptr(C), ld, ptr(A), K, ptr(B), ld, M, N, K, -1.0, sh),
                                              "dgemm"))
            print(f"dgemm f64 M={M} N={N} K={K}: {dt * 1e6:8.1f} us  {2 * M * N * K / dt * 1e-12:6.1f} TFLOP/s",
                  flush=True)
    if what in ("f64acc", "all"):
        # the C read's share: C += A B against C = A B (C not read) at the LU's trailing-update shapes
        for M, N, K in [(8192, 8192, 256), (8192, 8192, 128), (4096, 4096, 256), (4096, 4096, 128)]:
            ld = N + 2
            C = torch.randn(M, ld, dtype=torch.float64, device=dev)
            A = torch.randn(M, K, dtype=torch.float64, device=dev)
            B = torch.randn(K, ld, dtype=torch.float64, device=dev)
            for acc in (1, 0):
                dt = timeit(lambda: _native.check(lib.gelim_gpu_dgemm_ex(ptr(C), ld, ptr(A), K, ptr(B), ld, M, N, K,
                                                                         -1.0, acc, 0, sh), "dgemm_ex"))
                print(f"dgemm f64 M={M} N={N} K={K} accumulate={acc}: {dt * 1e6:8.1f} us  "
                      f"{2 * M * N * K / dt * 1e-12:6.1f} TFLOP/s", flush=True)
    if what in ("f32", "all"):
        for n in (2048, 4096, 8192, 16384):
            A = torch.randn(n, n, device=dev)
            B = torch.randn(n, n, device=dev)
            C = torch.empty(n, n, device=dev)
            dt = timeit(lambda: _native.check(lib.gelim_gpu_matmul_f32_ex(ptr(A), n, ptr(B), n, ptr(C), n, n, n, n, 0,
                                                                          _native.MM_MFMA if hasattr(_native, "MM_MFMA")
                                                                          else 2, sh), "mm"), reps=5)
            print(f"sgemm f32 n={n}: {dt * 1e6:9.1f} us  {2 * n ** 3 / dt * 1e-12:6.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
