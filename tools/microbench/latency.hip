// Latency microbenchmarks for the panel's per-column critical path on gfx950:
// workgroup barrier, LDS publish->barrier->read round trip, DPP max ladder,
// fp64 reciprocal, readlane.  One workgroup; thread 0 reports shader cycles
// per iteration (s_memtime).  Build: hipcc --offload-arch=gfx950 -O3 latency.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ unsigned dpp_shr(unsigned v, int) { return v; }

template <int CTRL, int RM>
__device__ __forceinline__ unsigned dpp(unsigned old, unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)v, CTRL, RM, 0xf, false);
}

__device__ __forceinline__ unsigned wave_max(unsigned v) {
  v = max(v, dpp<0x111, 0xf>(0u, v));
  v = max(v, dpp<0x112, 0xf>(0u, v));
  v = max(v, dpp<0x114, 0xf>(0u, v));
  v = max(v, dpp<0x118, 0xf>(0u, v));
  v = max(v, dpp<0x142, 0xa>(0u, v));
  v = max(v, dpp<0x143, 0xc>(0u, v));
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

template <int mode>
__global__ void bench(int iters, unsigned long long* out, double* sink) {
  __shared__ double buf[2][8][16];
  __shared__ uint64_t keys[2][8];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double acc = (double)t * 1e-3 + 1.0;
  unsigned v = t * 2654435761u;
  __syncthreads();
  const unsigned long long t0 = clk();
#pragma unroll 8
  for (int it = 0; it < iters; ++it) {
    const int par = it & 1;
    if constexpr (mode == 0) {  // bare barrier
      __syncthreads();
    } else if constexpr (mode == 1) {  // lane 0 of each wave publishes a key, barrier, everyone reads 8 keys
      if (lane == 0) keys[par][wave] = (uint64_t)v + wave;
      __syncthreads();
      uint64_t k = keys[par][lane & 7];
      v ^= (unsigned)k;
    } else if constexpr (mode == 2) {  // + one lane writes a 16-double row, all read it back
      if (lane == 0) keys[par][wave] = (uint64_t)v + wave;
      if (t == (it & 511)) {
#pragma unroll
        for (int c = 0; c < 16; c += 2)
          *reinterpret_cast<double2*>(&buf[par][wave][c]) = make_double2(acc, acc + c);
      }
      __syncthreads();
      uint64_t k = keys[par][lane & 7];
      const int pw = (int)(k & 7);
      double s = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) s += buf[par][pw][c];
      acc += s * 1e-9;
      v ^= (unsigned)k;
    } else if constexpr (mode == 3) {  // DPP max ladder + readlane (dependent chain)
      v = wave_max(v) + t;
    } else if constexpr (mode == 4) {  // fp64 IEEE reciprocal chain
      acc = 1.0 / (acc + 1.0);
    } else if constexpr (mode == 5) {  // dependent fp64 FMA chain
      acc = fma(acc, 0.999, 1e-3);
    } else if constexpr (mode == 6) {  // ballot + popcount + branch
      const uint64_t b = __ballot((v & 1) != 0);
      v += __popcll(b) + t;
    } else if constexpr (mode == 7) {  // LDS store -> load round trip within one wave
      buf[par][wave][lane & 15] = acc;
      __builtin_amdgcn_s_waitcnt(0);
      acc = buf[par][wave][(lane + 1) & 15] * 0.5 + 1.0;
    }
  }
  const unsigned long long t1 = clk();
  if (t == 0) out[mode] = (t1 - t0) / (unsigned long long)iters;
  if (acc == 12345.0 || v == 77u) sink[t] = acc + v;
}

__global__ void clock_ratio(unsigned long long* out, double* sink) {
  unsigned long long r0, r1;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r0)::"memory");
  const unsigned long long c0 = clk();
  double acc = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) acc = fma(acc, 0.999999, 1e-7);
  const unsigned long long c1 = clk();
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r1)::"memory");
  if (threadIdx.x == 0) {
    out[0] = c1 - c0;
    out[1] = r1 - r0;
  }
  if (acc == 1.2345) sink[0] = acc;
}

// dependent global-load chain over a buffer (next index stored in the data)
__global__ void chase(const int* __restrict__ nxt, int steps, unsigned long long* out, int* sink) {
  int i = 0;
  const unsigned long long t0 = clk();
  for (int s = 0; s < steps; ++s) i = nxt[i];
  const unsigned long long t1 = clk();
  if (threadIdx.x == 0) out[0] = (t1 - t0) / steps;
  if (i == -7) sink[0] = i;
}

// store by one workgroup, then the same thread reads it back after s_waitcnt
__global__ void store_load(int* buf, int steps, unsigned long long* out) {
  int v = 1;
  const unsigned long long t0 = clk();
  for (int s = 0; s < steps; ++s) {
    buf[(s * 64) & 0xffff] = v;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    v = __builtin_nontemporal_load(&buf[(s * 64) & 0xffff]) + 1;
  }
  const unsigned long long t1 = clk();
  if (threadIdx.x == 0) out[0] = (t1 - t0) / steps;
  if (v == -7) buf[1] = v;
}

int main(int argc, char** argv) {
  unsigned long long* d;
  double* sink;
  hipMalloc(&d, 64 * 8);
  hipMalloc(&sink, 1024 * 8);
  const char* names[] = {"barrier", "key publish+barrier+read", "row publish+barrier+read",
                         "DPP max ladder+readlane", "fp64 1/x", "fp64 fma chain",
                         "ballot+popc", "LDS st->ld (1 wave)"};
  for (int nt : {256, 512}) {
    for (int mode = 0; mode < 8; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        switch (mode) {
          case 0: hipLaunchKernelGGL(bench<0>, 1, nt, 0, 0, 4096, d, sink); break;
          case 1: hipLaunchKernelGGL(bench<1>, 1, nt, 0, 0, 4096, d, sink); break;
          case 2: hipLaunchKernelGGL(bench<2>, 1, nt, 0, 0, 4096, d, sink); break;
          case 3: hipLaunchKernelGGL(bench<3>, 1, nt, 0, 0, 4096, d, sink); break;
          case 4: hipLaunchKernelGGL(bench<4>, 1, nt, 0, 0, 4096, d, sink); break;
          case 5: hipLaunchKernelGGL(bench<5>, 1, nt, 0, 0, 4096, d, sink); break;
          case 6: hipLaunchKernelGGL(bench<6>, 1, nt, 0, 0, 4096, d, sink); break;
          default: hipLaunchKernelGGL(bench<7>, 1, nt, 0, 0, 4096, d, sink); break;
        }
      }
      hipDeviceSynchronize();
      unsigned long long h[64];
      hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
      printf("NT=%d %-28s %6llu cycles/iter\n", nt, names[mode], h[mode]);
    }
  }
  {
    // pointer chase: small (L2-resident) and large (HBM) footprints, 4 KiB stride
    for (size_t bytes : {(size_t)1 << 20, (size_t)1 << 30}) {
      const size_t n = bytes / 4;
      int* h = (int*)malloc(bytes);
      const size_t stride = 1024 + 16;  // ints
      for (size_t i = 0; i < n; ++i) h[i] = (int)((i + stride * 7) % n);
      int* dn;
      hipMalloc(&dn, bytes);
      hipMemcpy(dn, h, bytes, hipMemcpyHostToDevice);
      for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(chase, 1, 64, 0, 0, dn, 2000, d, (int*)sink);
      hipDeviceSynchronize();
      unsigned long long r;
      hipMemcpy(&r, d, 8, hipMemcpyDeviceToHost);
      printf("dependent global load, %zu MiB footprint: %llu cycles\n", bytes >> 20, r);
      hipFree(dn);
      free(h);
    }
    int* sb;
    hipMalloc(&sb, 1 << 20);
    hipLaunchKernelGGL(store_load, 1, 64, 0, 0, sb, 2000, d);
    hipDeviceSynchronize();
    unsigned long long r;
    hipMemcpy(&r, d, 8, hipMemcpyDeviceToHost);
    printf("store + vmcnt(0) + nontemporal load round trip: %llu cycles\n", r);
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(clock_ratio, 1, 64, 0, 0, d, sink);
    hipDeviceSynchronize();
    unsigned long long h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("s_memtime %llu cycles over %llu realtime ticks (100 MHz) -> %.3f GHz\n", h[0], h[1],
           (double)h[0] / (double)h[1] * 0.1);
  }
  return 0;
}
