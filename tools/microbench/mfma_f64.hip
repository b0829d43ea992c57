// fp64 matrix-core rate on gfx950: back-to-back v_mfma_f64_16x16x4_f64 with
// 4 independent accumulators per wave, one and two waves per SIMD, every CU.
// Prints cycles per MFMA per SIMD (s_memtime, shader clock) and the chip-wide
// TFLOP/s from hipEvent wall time.  This is the number the fp64 trailing GEMM
// (csrc/hip/dgemm.hip) is priced against.
//
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/mfma_f64.hip -o tools/microbench/mfma_f64
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

template <int NACC>
__global__ void mfma_loop(double* out, unsigned long long* cyc, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{seed, seed * 0.5, seed * 0.25, seed * 0.125};
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC>
void run(int threads, int blocks, int iters) {
  double* out;
  unsigned long long* cyc;
  CHECK(hipMalloc(&out, sizeof(double) * threads * blocks));
  CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1.0);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(mfma_loop<NACC>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1.0);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long h[1];
  CHECK(hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost));
  const double waves = (double)blocks * threads / 64;
  const double flops = waves * iters * NACC * 2.0 * 16 * 16 * 4;
  const int wps = threads / 256;  // waves per SIMD at one block per CU
  std::printf("acc=%d waves/SIMD=%d blocks=%d: %.1f cycles per MFMA per wave (s_memtime), "
              "%.1f per SIMD, %.2f TFLOP/s wall\n",
              NACC, wps > 0 ? wps : 1, blocks, (double)h[0] / (iters * NACC),
              (double)h[0] / (iters * NACC) / (wps > 0 ? wps : 1), flops / (ms * 1e-3) / 1e12);
  CHECK(hipFree(out));
  CHECK(hipFree(cyc));
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  std::printf("%s, %d CUs\n", p.gcnArchName, p.multiProcessorCount);
  const int cus = p.multiProcessorCount;
  run<4>(256, cus, 20000);
  run<8>(256, cus, 10000);
  run<4>(512, cus, 10000);
  run<8>(512, cus, 10000);
  return 0;
}
