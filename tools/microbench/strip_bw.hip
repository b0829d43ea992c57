// Strip-read bandwidth: one workgroup (512 threads) streams an m x 16 fp64
// strip whose rows are `ld` doubles apart (ld = 2056: a column strip of a
// row-major 2048^2 matrix; ld = 16: strip-major storage), with the MFMA-tile
// access pattern of the trailing update (lane: row q+4r, column l&15).
// Also: 128 workgroups at once on disjoint strips (the wide update).
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ __launch_bounds__(512) void strip_read(const double* __restrict__ A, long ld, long strip_stride,
                                                  int m, double* __restrict__ out, unsigned long long* cyc) {
  const double* S = A + blockIdx.x * strip_stride;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  double acc = 0.0;
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  const int nblk = m / 16;
  for (int b0 = wave; b0 < nblk; b0 += 8 * 4) {
    double v[4][4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = min(16 * (b0 + 8 * s) + q + 4 * r, m - 1);
        v[s][r] = S[(long)row * ld + r16];
      }
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc += v[s][r];
  }
  __syncthreads();
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (t == 0 && blockIdx.x == 0) *cyc = t1 - t0;
  if (acc == 1.2345) out[t] = acc;
}

int main() {
  const int n = 2048;
  const long ldr = 2056;
  double* A;
  double* out;
  unsigned long long* cyc;
  hipMalloc(&A, sizeof(double) * n * ldr + (1 << 20));
  hipMalloc(&out, 4096 * 8);
  hipMalloc(&cyc, 8);
  hipMemset(A, 0, sizeof(double) * n * ldr);
  struct Cfg { const char* name; long ld; long stride; int blocks; };
  Cfg cfgs[] = {{"row-major strip (ld 2056), 1 WG", ldr, 16, 1},
                {"strip-major (ld 16), 1 WG", 16, 16L * n, 1},
                {"row-major strips, 128 WGs", ldr, 16, 128},
                {"strip-major, 128 WGs", 16, 16L * n, 128}};
  for (auto& c : cfgs) {
    float best = 1e9f;
    unsigned long long hc = 0;
    for (int rep = 0; rep < 5; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(strip_read, c.blocks, 512, 0, 0, A, c.ld, c.stride, n, out, cyc);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
      hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost);
    }
    const double bytes = (double)n * 16 * 8 * c.blocks;
    printf("%-36s kernel %.2f us (wg0 %llu cycles = %.2f us)  %.1f GB/s aggregate\n", c.name, best * 1e3,
           hc, hc / 2400.0, bytes / (best * 1e-3) * 1e-9);
  }
  return 0;
}
