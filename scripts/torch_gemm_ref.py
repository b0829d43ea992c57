"""fp64 C -= A B through torch (rocBLAS / hipBLASLt) at the shapes of scripts/gemm_bench.py, for comparison
with gelim's MFMA GEMM.  python scripts/torch_gemm_ref.py"""
import torch, time
d = torch.device("cuda:0")
for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 256), (4096, 4096, 256)]:
    A = torch.randn(M, K, dtype=torch.float64, device=d); B = torch.randn(K, N, dtype=torch.float64, device=d)
    C = torch.randn(M, N, dtype=torch.float64, device=d)
    for _ in range(3): C.addmm_(A, B, alpha=-1.0)
    torch.cuda.synchronize(); t = time.perf_counter(); r = 10
    for _ in range(r): C.addmm_(A, B, alpha=-1.0)
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / r
    print(f"torch addmm f64 M={M} N={N} K={K}: {dt*1e6:.1f} us {2*M*N*K/dt/1e12:.1f} TFLOP/s")
