// Where the time of an 8-workgroup fused chain kernel went (round 6): the
// first form of DistributedRBT's W = Dinv B; D -= L W kernel (16-column
// strips, 512 threads, every workgroup streaming all of Dinv and L through
// LDS), with s_memtime stamps per wave, plus a dependent-accumulator
// v_mfma_f64_16x16x4f64 chain.  Result (profiles/dist_rbt_replay_r6.md):
// 15.8 k cycles to ISSUE the loads, 20.8 k in the chunk loop -- the load path
// of one CU, not its matrix core, bound it; the executor now runs these
// products as one wave per 16 x 16 tile (csrc/hip/drbt_exec.hip).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/microbench/chain_stamps.hip -o /tmp/chain_stamps
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
namespace gelim { namespace dev { typedef double d4 __attribute__((ext_vector_type(4))); } }
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1);} } while (0)
constexpr int kChainThreads = 512;

template <bool kW>
__global__ __launch_bounds__(kChainThreads) void drbt_chain_kernel(const double* __restrict__ Dk,
                                                                   const double* __restrict__ B,
                                                                   double* __restrict__ W,
                                                                   const double* __restrict__ L,
                                                                   double* __restrict__ D, unsigned long long* st, int mode) {
  constexpr int NBk = 128, KC = 32, SA = 36, NCH = (kW ? 2 : 1) * NBk / KC;  // chunks: Dk's then L's
  constexpr int PER = NBk * KC / 2 / kChainThreads;                          // double2 per thread per chunk
  __shared__ __attribute__((aligned(16))) double as[2][NBk * SA];
  __shared__ __attribute__((aligned(16))) double bs[kW ? NBk * 16 : 1];  // the B strip (stage 1)
  __shared__ __attribute__((aligned(16))) double wl[NBk * 16];           // the W strip
  unsigned long long T0 = __builtin_amdgcn_s_memtime();
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int c0 = blockIdx.x * 16, r16 = lane & 15, q = lane >> 4, R0 = 16 * wave;

  // every global load of the launch, in the order they are consumed
  constexpr int SP = NBk * 16 / 2 / kChainThreads;  // double2 of the strip per thread
  double2 ch[NCH][PER], sv[SP];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const double* src = (kW && c < NBk / KC) ? Dk : L;
    const int kc = KC * (c % (NBk / KC));
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kChainThreads * i, row = e >> 4, col = 2 * (e & 15);
      ch[c][i] = *reinterpret_cast<const double2*>(src + (int64_t)row * NBk + kc + col);
    }
    if (c == 0) {  // the strip the first chunks multiply
      const double* sp = kW ? B : W;
#pragma unroll
      for (int i = 0; i < SP; ++i) {
        const int e = t + kChainThreads * i, row = e >> 3, col = 2 * (e & 7);
        sv[i] = *reinterpret_cast<const double2*>(sp + (int64_t)row * NBk + c0 + col);
      }
    }
  }
  gelim::dev::d4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = D[(int64_t)(R0 + q + 4 * r) * NBk + c0 + r16];
  __builtin_amdgcn_sched_barrier(0);

  auto stage = [&](int buf, int c) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = t + kChainThreads * i, row = e >> 4, col = 2 * (e & 15);
      *reinterpret_cast<double2*>(&as[buf][row * SA + col]) = ch[c][i];
    }
  };
  unsigned long long T1 = __builtin_amdgcn_s_memtime();
  stage(0, 0);
#pragma unroll
  for (int i = 0; i < SP; ++i) {
    const int e = t + kChainThreads * i, row = e >> 3, col = 2 * (e & 7);
    *reinterpret_cast<double2*>((kW ? bs : wl) + row * 16 + col) = sv[i];
  }
  __syncthreads();
  unsigned long long T2 = __builtin_amdgcn_s_memtime();
  gelim::dev::d4 w = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const double* a_s = as[c & 1] + (R0 + r16) * SA + q;
    const bool first = kW && c < NBk / KC;  // W = Dk B (else D -= L W)
    const int kc = KC * (c % (NBk / KC));
    const double* b_s = (first ? bs : wl) + (kc + q) * 16 + r16;
#pragma unroll
    for (int s = 0; s < KC / 4; ++s) {
      const double av = a_s[4 * s], bv = b_s[64 * s];
      if (first)
        w = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, w, 0, 0, 0);
      else
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-av, bv, acc, 0, 0, 0);
    }
    if (kW && c == NBk / KC - 1) {  // W's tile: to LDS for the update, to global for the rest
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        wl[(R0 + q + 4 * r) * 16 + r16] = w[r];
        W[(int64_t)(R0 + q + 4 * r) * NBk + c0 + r16] = w[r];
      }
    }
    if (c + 1 < NCH) stage((c + 1) & 1, c + 1);
    __syncthreads();
  }
  unsigned long long T3 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int r = 0; r < 4; ++r) D[(int64_t)(R0 + q + 4 * r) * NBk + c0 + r16] = acc[r];
  if (lane == 0) { unsigned long long* o = st + (blockIdx.x * 8 + wave) * 4; o[0] = T0; o[1] = T1; o[2] = T2; o[3] = T3; }
}


__global__ void dep_chain(double* out, unsigned long long* cyc, int iters) {
  gelim::dev::d4 acc = {1.0, 0.5, 0.25, 0.125};
  double a = 1.0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-3;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  double *buf; unsigned long long* st;
  CHECK(hipMalloc(&buf, 8 * 128 * 128 * 8));
  CHECK(hipMemset(buf, 0, 8 * 128 * 128 * 8));
  CHECK(hipMalloc(&st, 8 * 8 * 4 * 8));
  double *Dk = buf, *B = buf + 16384, *W = buf + 2 * 16384, *L = buf + 3 * 16384, *D = buf + 4 * 16384;
  for (int v = 0; v < 2; ++v) {
    for (int rep = 0; rep < 5; ++rep) {
      if (v == 0) hipLaunchKernelGGL(drbt_chain_kernel<true>, dim3(8), dim3(512), 0, 0, Dk, B, W, L, D, st, 0);
      else hipLaunchKernelGGL(drbt_chain_kernel<false>, dim3(8), dim3(512), 0, 0, Dk, B, W, L, D, st, 0);
      CHECK(hipDeviceSynchronize());
    }
    unsigned long long h[8 * 8 * 4];
    CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
    double s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 64; ++i) { s1 += h[4*i+1] - h[4*i]; s2 += h[4*i+2] - h[4*i+1]; s3 += h[4*i+3] - h[4*i+2]; }
    std::printf("variant %s: cycles issue-loads %.0f, wait+stage0+barrier %.0f, chunk loop %.0f (avg over waves)\n", v ? "D only" : "W + D", s1 / 64, s2 / 64, s3 / 64);
  }
  unsigned long long c; double* o; CHECK(hipMalloc(&o, 4096)); unsigned long long* cy; CHECK(hipMalloc(&cy, 64));
  hipLaunchKernelGGL(dep_chain, dim3(1), dim3(64), 0, 0, o, cy, 10000); CHECK(hipDeviceSynchronize());
  hipLaunchKernelGGL(dep_chain, dim3(1), dim3(64), 0, 0, o, cy, 10000); CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost));
  std::printf("dependent f64 16x16x4 chain, one wave: %.1f cycles per MFMA\n", c / 10000.0);
  hipLaunchKernelGGL(dep_chain, dim3(1), dim3(512), 0, 0, o, cy, 10000); CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(&c, cy, 8, hipMemcpyDeviceToHost));
  std::printf("dependent f64 16x16x4 chain, 8 waves on one CU: %.1f cycles per MFMA per wave\n", c / 10000.0);
  return 0;
}
