// Back substitution U x = y on the GPU (the reference's solveGauss,
// Pthreads/Version-1/gauss_internal_input.c:212-227, a serial O(n^2) loop
// there).
//
// Default: ONE persistent launch (backsub_persist_kernel).  Row block b (64
// equations) belongs to workgroup b and x is produced bottom-up.  Every
// workgroup preloads its 64x64 diagonal triangle into wave 0's registers,
// then takes the solved x blocks below it in order (last block first): for
// each it prefetches the matching 64x64 block of U BEFORE polling that
// block's flag, so after the hand-off only x_c (512 B) is read, and
// subtracts U[b, c] x_c (wave per row, shuffle sums).  After the last one,
// wave 0 solves the triangle (rows in lanes, x_i broadcast with v_readlane:
// mul -> readlane -> fma per step) and publishes x_b (sc1 stores, drain,
// flag).  The critical path per block is one hand-off + one block mat-vec +
// the 64-step chain, instead of one dependent kernel launch per block.
// Spins are bounded (200 ms) and report through an error word.
//
// Rows may be indirect: perm[i] is the row of U (and of y) that holds
// equation i -- the resident LU (rlu.hip) leaves U rows at their physical
// positions.  Without perm, row i is equation i.
//
// Fallback when the blocks cannot all be resident (more than 256 blocks,
// n > 16384): one launch per block (backsub_step_kernel).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kBS = 64;
constexpr int kMaxPersistBlocks = 256;
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

// Row of equation i; a row map entry outside [0, n) (a corrupt map, e.g. one
// left stale by an aborted factorisation) is clamped, never dereferenced --
// the persistent kernel reports it through its error word (code 7).
__device__ __forceinline__ int rowof(const int* perm, int i, int n) {
  return perm ? min(max(perm[i], 0), n - 1) : i;
}

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <typename T>
__global__ void copy_y_kernel(const T* __restrict__ U, int64_t ldu, const T* __restrict__ y,
                              int64_t incy, const int* __restrict__ perm, double* __restrict__ yw,
                              double* __restrict__ bnorm, int n, int unit) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = rowof(perm, i, n);
  const double v = (double)y[(int64_t)r * incy];
  yw[i] = v;
  if (bnorm) bnorm[i] = unit ? v : v / (double)U[(int64_t)r * ldu + i];
}

// Wave 0's copy of a diagonal block: lane l keeps equation i0+l's row
// (columns i0..i0+nb) and the reciprocal of its diagonal.
template <typename T>
__device__ __forceinline__ void load_diag(const T* __restrict__ U, int64_t ldu, const int* perm, int n, int i0,
                                          int nb, int unit, double (&row)[kBS], double& rinv) {
  const int l = threadIdx.x & 63;
  const int lc = min(l, nb - 1);
  const T* src = U + (int64_t)rowof(perm, i0 + lc, n) * ldu + i0;
#pragma unroll
  for (int c = 0; c < kBS; ++c) row[c] = dev::load_sel(src + min(c, nb - 1), l < nb && c < nb);
  rinv = unit ? 1.0 : 1.0 / (double)src[lc];
}

// One wave solves the nb x nb triangle: x_i broadcast with v_readlane (i is
// wave-uniform), so the serial chain is mul -> readlane -> fma per step.
__device__ __forceinline__ double solve_diag(const double (&row)[kBS], double rinv, double yv, int nb) {
  const int l = threadIdx.x & 63;
  double xv = 0.0;
#pragma unroll
  for (int i = kBS - 1; i >= 0; --i) {
    if (i < nb) {
      const double xi_l = yv * rinv;  // meaningful in lane i only
      const uint64_t b = __builtin_bit_cast(uint64_t, xi_l);
      const double xi = __builtin_bit_cast(
          double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), i) << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)b, i));
      if (l == i) xv = xi;
      yv = (l < i) ? fma(-row[i], xi, yv) : yv;
    }
  }
  return xv;
}

// Bounded poll of flag c by lane 0 of the calling wave (wave-uniform result).
__device__ __forceinline__ bool poll_flag(unsigned* flags, int c, int* err, bool nap) {
  int good = 1;
  if (__lane_id() == 0) {
    if (__hip_atomic_load(&flags[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      const unsigned long long t0 = rtc();
      while (__hip_atomic_load(&flags[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || rtc() - t0 > kSpinTicks) {
          __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          good = 0;
          break;
        }
        if (nap) __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  return __builtin_amdgcn_readfirstlane(good) != 0;  // lane 0's verdict (no ds_bpermute round trip)
}

// acc -= U[rows of this block, block c] . x_c, row = lane: the U block was
// prefetched into u[] before the poll; x_c (stored write-through by its
// producer) is read with one agent-scope load per lane and broadcast with
// readlane.
template <typename T>
__device__ __forceinline__ bool apply_block(const T* __restrict__ U, int64_t ldu, int pr, int c, int n,
                                            const double* __restrict__ x, unsigned* flags, int* err, bool nap,
                                            double& acc) {
  const int lane = __lane_id();
  const int c0 = c * kBS, cw = min(kBS, n - c0);
  double u[kBS];
  const T* urow = U + (int64_t)pr * ldu + c0;
#pragma unroll
  for (int k = 0; k < kBS; ++k) u[k] = (double)urow[min(k, cw - 1)];
  if (!poll_flag(flags, c, err, nap)) return false;
  const double xl = __builtin_bit_cast(
      double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(x + c0 + min(lane, cw - 1)),
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint64_t xb = __builtin_bit_cast(uint64_t, xl);
  const int xlo = (int)(unsigned)xb, xhi = (int)(unsigned)(xb >> 32);
#pragma unroll
  for (int k = 0; k < kBS; ++k) {
    if (k < cw) {
      const double xk = __builtin_bit_cast(double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane(xhi, k) << 32) |
                                                        (unsigned)__builtin_amdgcn_readlane(xlo, k));
      acc = fma(-u[k], xk, acc);
    }
  }
  return true;
}

// Block b (64 equations, lane = equation) of the persistent back
// substitution.  Wave 0 owns the critical path: it keeps the diagonal
// triangle in registers, takes the LAST hand-off (block b+1) itself and then
// solves the triangle; waves 1..3 take the blocks below b+1 (their x are
// published earlier) round-robin in the background and hand their partial
// sums over through LDS behind one barrier.  Every load of a U block is
// issued before its flag is polled.
template <typename T>
__global__ __launch_bounds__(256) void backsub_persist_kernel(const T* __restrict__ U, int64_t ldu,
                                                              const T* __restrict__ y, int64_t incy,
                                                              const int* __restrict__ perm,
                                                              double* __restrict__ x,
                                                              double* __restrict__ bnorm, int n,
                                                              int unit, unsigned* flags, int* err) {
  __shared__ double part[4][kBS];
  const int b = blockIdx.x, nb = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int r0 = b * kBS, rows = min(kBS, n - r0);
  const int i = r0 + min(lane, rows - 1);
  const int pr = rowof(perm, i, n);
  if (wv == 0 && perm && lane < rows && perm[i] != pr)
    __hip_atomic_store(err, 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double acc = 0.0;
  bool ok = true;
  if (wv == 0) {
    double drow[kBS];
    double rinv = 1.0;
    load_diag<T>(U, ldu, perm, n, r0, rows, unit, drow, rinv);
    const double v = (double)y[(int64_t)pr * incy];
    if (bnorm && lane < rows) bnorm[i] = unit ? v : v / (double)U[(int64_t)pr * ldu + i];
    if (b + 1 < nb) ok = apply_block<T>(U, ldu, pr, b + 1, n, x, flags, err, false, acc);
    __syncthreads();
    if (!ok) return;
    double yv = v + acc + part[1][lane] + part[2][lane] + part[3][lane];
    const double xv = solve_diag(drow, rinv, yv, rows);
    if (lane < rows)
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + r0 + lane), __builtin_bit_cast(unsigned long long, xv),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(&flags[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // background waves: blocks nb-1 .. b+2, wave 1 + (nb-1-c) % 3
  for (int c = nb - 1 - (wv - 1); c >= b + 2 && ok; c -= 3)
    ok = apply_block<T>(U, ldu, pr, c, n, x, flags, err, true, acc);
  part[wv][lane] = acc;  // 0 when the wave had no block
  __syncthreads();
}

// ---- fallback: one launch per block ----------------------------------------

template <typename T>
__global__ __launch_bounds__(64) void diag_solve_kernel(const T* __restrict__ U, int64_t ldu,
                                                        const int* __restrict__ perm,
                                                        double* __restrict__ yw,
                                                        double* __restrict__ x, int i0, int nb,
                                                        int unit, int n) {
  double row[kBS];
  double rinv;
  load_diag<T>(U, ldu, perm, n, i0, nb, unit, row, rinv);
  const int l = threadIdx.x & 63;
  const double xv = solve_diag(row, rinv, dev::load_sel(yw + i0 + min(l, nb - 1), l < nb), nb);
  if (l < nb) x[i0 + l] = xv;
}

// Every workgroup subtracts block [i0, i0+nb)'s solved x from its rows above
// (wave per row); workgroup 0 owns the 64 rows right above the block and,
// once they are final, solves that diagonal block too.
template <typename T>
__global__ __launch_bounds__(256) void backsub_step_kernel(const T* __restrict__ U, int64_t ldu,
                                                           const int* __restrict__ perm,
                                                           double* __restrict__ yw,
                                                           double* __restrict__ x, int i0, int nb,
                                                           int unit, int n) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int p0 = i0 > kBS ? i0 - kBS : 0;  // the next diagonal block [p0, i0)
  const double xl = dev::load_sel(x + i0 + min(lane, nb - 1), lane < nb);
  if (blockIdx.x == 0) {
    constexpr int kRows = kBS / 4;
    double v[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      v[k] = dev::load_sel(U + (int64_t)rowof(perm, min(r, i0 - 1), n) * ldu + i0 + min(lane, nb - 1),
                           lane < nb && r < i0) * xl;
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      const double sum = dev::wave_sum(v[k]);
      if (lane == 0 && r < i0) yw[r] -= sum;
    }
    __syncthreads();
    if (wv == 0) {
      double row[kBS];
      double rinv;
      load_diag<T>(U, ldu, perm, n, p0, i0 - p0, unit, row, rinv);
      const int l = lane;
      const double xv = solve_diag(row, rinv, dev::load_sel(yw + p0 + min(l, i0 - p0 - 1), l < i0 - p0), i0 - p0);
      if (l < i0 - p0) x[p0 + l] = xv;
    }
    return;
  }
  const int nw = (gridDim.x - 1) * 4;
  for (int r = (blockIdx.x - 1) * 4 + wv; r < p0; r += nw) {
    double v = dev::load_sel(U + (int64_t)rowof(perm, r, n) * ldu + i0 + min(lane, nb - 1), lane < nb) * xl;
    v = dev::wave_sum(v);
    if (lane == 0) yw[r] -= v;
  }
}

template <typename T>
int backsub_impl(const T* U, int64_t ldu, const T* y, int64_t incy, double* x, double* bnorm,
                 int64_t n, int unit, double* yw, hipStream_t s, const int* perm, int* err) {
  const int64_t nblk = (n + kBS - 1) / kBS;
  // the persistent form needs every block resident (flag hand-offs);
  // checked once per (type, block count)
  bool persist = nblk <= kMaxPersistBlocks;
  if (persist) {
    int per = 0;
    persist = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, backsub_persist_kernel<T>, 256, 0) == hipSuccess &&
              coresident(per, nblk);
  }
  if (persist) {
    // flags (+ the error word when the caller has none) live in yw
    unsigned* flags = reinterpret_cast<unsigned*>(yw);
    int* e = err ? err : reinterpret_cast<int*>(flags + nblk);
    // (nblk + 1) words always fit in yw's n doubles; round to 16 bytes when
    // that still fits (a 16-byte multiple is the fast memset path)
    const size_t bytes = ((size_t)nblk + 1) * 4;
    const size_t rounded = (bytes + 15) / 16 * 16;
    GELIM_TRY(zero_async(flags, rounded <= (size_t)n * sizeof(double) ? rounded : bytes, s));
    hipLaunchKernelGGL(backsub_persist_kernel<T>, dim3((unsigned)nblk), dim3(256), 0, s, U, ldu, y, incy,
                       perm, x, bnorm, (int)n, unit, flags, e);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  hipLaunchKernelGGL(copy_y_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U, ldu, y, incy,
                     perm, yw, bnorm, (int)n, unit);
  HIP_TRY(hipGetLastError());
  int64_t i0 = (n - 1) / kBS * kBS;
  hipLaunchKernelGGL(diag_solve_kernel<T>, dim3(1), dim3(64), 0, s, U, ldu, perm, yw, x, (int)i0,
                     (int)(n - i0), unit, (int)n);
  HIP_TRY(hipGetLastError());
  for (int64_t i1 = n; i0 > 0; i1 = i0, i0 -= kBS) {
    const int nb = (int)(i1 - i0);
    const int64_t rows = i0 > kBS ? i0 - kBS : 0;  // rows above the next block
    const int blocks = 1 + (int)std::min<int64_t>((rows + 3) / 4, 1024);
    hipLaunchKernelGGL(backsub_step_kernel<T>, dim3(blocks), dim3(256), 0, s, U, ldu, perm, yw, x,
                       (int)i0, nb, unit, (int)n);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

}  // namespace

int backsub_f64(const double* U, int64_t ldu, const double* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s, const int* perm,
                int* err) {
  return backsub_impl<double>(U, ldu, y, incy, x, bnorm, n, unit, yw, s, perm, err);
}

int backsub_f32(const float* U, int64_t ldu, const float* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s, const int* perm,
                int* err) {
  return backsub_impl<float>(U, ldu, y, incy, x, bnorm, n, unit, yw, s, perm, err);
}

}  // namespace gelim

extern "C" int gelim_gpu_backsub(const double* dU, int64_t ldu, const double* dy, int64_t incy,
                                 double* dx, double* dbnorm, int64_t n, int unit, void* stream) {
  if (n <= 0) return GELIM_FAIL(GELIM_E_ARG, "backsub: n <= 0");
  hipStream_t s = (hipStream_t)stream;
  double* yw = nullptr;
  HIP_TRY(hipMallocAsync((void**)&yw, sizeof(double) * (n + 2), s));
  int rc = gelim::backsub_f64(dU, ldu, dy, incy, dx, dbnorm, n, unit, yw, s, nullptr, nullptr);
  HIP_TRY(hipFreeAsync(yw, s));
  return rc;
}
