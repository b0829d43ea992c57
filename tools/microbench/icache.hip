// Instruction-cache microbenchmark: the same instruction stream executed as
// straight-line code (template-unrolled, ~KB .. 256 KB of code) and as a
// rolled loop (one body in the cache).  One wave per workgroup, 32 or 256
// workgroups (one per CU), shader cycles per instruction from s_memtime.
//
// Why: the leaf (biglu.hip) and fused step (lu_panel.hip) kernels unroll
// their column loops at compile time (register-resident panels), which makes
// them 150-240 KB of straight-line code executed once per launch.
//
//   hipcc --offload-arch=gfx950 -O3 -o icache icache.hip && ./icache
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// 32 independent v_fma_f64 on 8 accumulators: 256 bytes of code
#define FMA8                                                                    \
  "v_fma_f64 v[0:1], v[16:17], v[18:19], v[0:1]\n"                              \
  "v_fma_f64 v[2:3], v[16:17], v[18:19], v[2:3]\n"                              \
  "v_fma_f64 v[4:5], v[16:17], v[18:19], v[4:5]\n"                              \
  "v_fma_f64 v[6:7], v[16:17], v[18:19], v[6:7]\n"                              \
  "v_fma_f64 v[8:9], v[16:17], v[18:19], v[8:9]\n"                              \
  "v_fma_f64 v[10:11], v[16:17], v[18:19], v[10:11]\n"                          \
  "v_fma_f64 v[12:13], v[16:17], v[18:19], v[12:13]\n"                          \
  "v_fma_f64 v[14:15], v[16:17], v[18:19], v[14:15]\n"
#define BODY asm volatile(FMA8 FMA8 FMA8 FMA8 ::: "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", \
                          "v10", "v11", "v12", "v13", "v14", "v15")

template <int N>
struct Straight {
  static __device__ __forceinline__ void run() {
    BODY;
    Straight<N - 1>::run();
  }
};
template <>
struct Straight<0> {
  static __device__ __forceinline__ void run() {}
};

template <int N>
__global__ __launch_bounds__(64) void straight_kernel(unsigned long long* cyc, int reps) {
  asm volatile("v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n v_mov_b32 v18, 0\n v_mov_b32 v19, 0" ::: "v16", "v17", "v18",
               "v19");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) Straight<N>::run();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int N>
__global__ __launch_bounds__(64) void loop_kernel(unsigned long long* cyc, int reps) {
  asm volatile("v_mov_b32 v16, 0\n v_mov_b32 v17, 0\n v_mov_b32 v18, 0\n v_mov_b32 v19, 0" ::: "v16", "v17", "v18",
               "v19");
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < reps; ++r) {
#pragma unroll 1
    for (int i = 0; i < N; ++i) BODY;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int N>
void run(int blocks) {
  unsigned long long* cyc;
  CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks));
  unsigned long long h[2];
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 2; ++rep) {  // second launch: warm L2
      if (k == 0) hipLaunchKernelGGL(straight_kernel<N>, dim3(blocks), dim3(64), 0, 0, cyc, 1);
      else hipLaunchKernelGGL(loop_kernel<N>, dim3(blocks), dim3(64), 0, 0, cyc, 1);
      CHECK(hipDeviceSynchronize());
    }
    CHECK(hipMemcpy(&h[k], cyc, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  }
  const double ins = 32.0 * N;
  std::printf("code %6d B, %3d WGs: straight %7.2f cycles/instr, loop %5.2f cycles/instr (%.1fx)\n", 256 * N, blocks,
              h[0] / ins, h[1] / ins, (double)h[0] / h[1]);
  CHECK(hipFree(cyc));
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  std::printf("%s, %d CUs\n", p.gcnArchName, p.multiProcessorCount);
  for (int b : {32, 256}) {
    run<16>(b);
    run<64>(b);
    run<128>(b);
    run<256>(b);
    run<512>(b);
    run<800>(b);
  }
  return 0;
}
