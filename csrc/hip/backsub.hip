// Back substitution U x = y on the GPU (the reference's solveGauss,
// Pthreads/Version-1/gauss_internal_input.c:212-227, which is a serial O(n^2)
// loop there).
//
// Blocked right-to-left: for each 64-row diagonal block (bottom-up)
//   diag kernel   : one wave64 solves the 64x64 triangle, the block staged in
//                   LDS, x_i broadcast across lanes with a shuffle;
//   update kernel : y[0:i0] -= U[0:i0, blk] x_blk, one wave per row,
//                   coalesced 512-byte row segments + shuffle reduction.
// A leading copy kernel gathers y (a strided column of the augmented matrix)
// into a contiguous work vector and optionally emits the reference's
// transformed B = y_i / U_ii (printed by VERIFY, P1i:292-295).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kBS = 64;

template <typename T>
__global__ void copy_y_kernel(const T* __restrict__ U, int64_t ldu, const T* __restrict__ y,
                              int64_t incy, double* __restrict__ yw, double* __restrict__ bnorm,
                              int n, int unit) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = (double)y[(int64_t)i * incy];
  yw[i] = v;
  if (bnorm) bnorm[i] = unit ? v : v / (double)U[(int64_t)i * ldu + i];
}

// One wave solves the nb x nb diagonal block at i0: lane l keeps row l in
// registers; x_i is broadcast with v_readlane (i is wave-uniform) — no LDS,
// no shuffles on the serial chain.
template <typename T>
__device__ __forceinline__ void diag_solve_wave(const T* __restrict__ U, int64_t ldu,
                                                double* __restrict__ yw, double* __restrict__ x,
                                                int i0, int nb, int unit) {
  const int l = threadIdx.x & 63;
  double row[kBS];
  const T* src = U + (int64_t)(i0 + min(l, nb - 1)) * ldu + i0;
#pragma unroll
  for (int c = 0; c < kBS; ++c) row[c] = (l < nb && c < nb) ? (double)src[min(c, nb - 1)] : 0.0;
  const int lc = min(l, nb - 1);
  double yv = dev::load_sel(yw + i0 + lc, l < nb);
  // reciprocal of every lane's own diagonal, computed in parallel up front:
  // the serial chain is then mul -> readlane -> fma per step
  const double dg = dev::load_sel(U + (int64_t)(i0 + lc) * ldu + i0 + lc, l < nb, T(1));
  const double rinv = unit ? 1.0 : 1.0 / dg;
  double xv = 0.0;
#pragma unroll
  for (int i = kBS - 1; i >= 0; --i) {
    if (i < nb) {
      const double xi_l = yv * rinv;  // meaningful in lane i only
      const double xi = __builtin_bit_cast(
          double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane(
                       (int)(__builtin_bit_cast(uint64_t, xi_l) >> 32), i)
                   << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(uint64_t, xi_l), i));
      if (l == i) xv = xi;
      yv = (l < i) ? fma(-row[i], xi, yv) : yv;
    }
  }
  if (l < nb) x[i0 + l] = xv;
}

template <typename T>
__global__ __launch_bounds__(64) void diag_solve_kernel(const T* __restrict__ U, int64_t ldu,
                                                        double* __restrict__ yw,
                                                        double* __restrict__ x, int i0, int nb,
                                                        int unit) {
  diag_solve_wave<T>(U, ldu, yw, x, i0, nb, unit);
}

// One launch per block (fused form of update_kernel + diag_solve_kernel):
// every workgroup subtracts block [i0, i0+nb)'s solved x from its rows above
// (wave per row); workgroup 0 owns the 64 rows right above the block and,
// once they are final, solves that diagonal block too, so the next launch
// can go on with it.
template <typename T>
__global__ __launch_bounds__(256) void backsub_step_kernel(const T* __restrict__ U, int64_t ldu,
                                                           double* __restrict__ yw,
                                                           double* __restrict__ x, int i0, int nb,
                                                           int unit) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int p0 = i0 > kBS ? i0 - kBS : 0;  // the next diagonal block [p0, i0)
  const double xl = dev::load_sel(x + i0 + min(lane, nb - 1), lane < nb);
  if (blockIdx.x == 0) {
    // the 64 rows [p0, i0): 16 per wave, every load in flight before the sums
    constexpr int kRows = kBS / 4;
    double v[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      v[k] = dev::load_sel(U + (int64_t)min(r, i0 - 1) * ldu + i0 + min(lane, nb - 1),
                           lane < nb && r < i0) * xl;
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      const double sum = dev::wave_sum(v[k]);
      if (lane == 0 && r < i0) yw[r] -= sum;
    }
    __syncthreads();
    if (wv == 0) diag_solve_wave<T>(U, ldu, yw, x, p0, i0 - p0, unit);
    return;
  }
  const int nw = (gridDim.x - 1) * 4;
  for (int r = (blockIdx.x - 1) * 4 + wv; r < p0; r += nw) {
    double v = dev::load_sel(U + (int64_t)r * ldu + i0 + min(lane, nb - 1), lane < nb) * xl;
    v = dev::wave_sum(v);
    if (lane == 0) yw[r] -= v;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void update_kernel(const T* __restrict__ U, int64_t ldu,
                                                     double* __restrict__ yw,
                                                     const double* __restrict__ x, int i0,
                                                     int nb) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  const double xl = (lane < nb) ? x[i0 + lane] : 0.0;
  for (int r = wave; r < i0; r += nwaves) {
    double v = (lane < nb) ? (double)U[(int64_t)r * ldu + i0 + lane] * xl : 0.0;
    v = dev::wave_sum(v);
    if (lane == 0) yw[r] -= v;
  }
}

template <typename T>
int backsub_impl(const T* U, int64_t ldu, const T* y, int64_t incy, double* x, double* bnorm,
                 int64_t n, int unit, double* yw, hipStream_t s) {
  hipLaunchKernelGGL(copy_y_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U, ldu,
                     y, incy, yw, bnorm, (int)n, unit);
  HIP_TRY(hipGetLastError());
  // last diagonal block, then one fused launch per block: update the rows
  // above with its x and solve the next diagonal block
  int64_t i0 = (n - 1) / kBS * kBS;
  hipLaunchKernelGGL(diag_solve_kernel<T>, dim3(1), dim3(64), 0, s, U, ldu, yw, x, (int)i0,
                     (int)(n - i0), unit);
  HIP_TRY(hipGetLastError());
  for (int64_t i1 = n; i0 > 0; i1 = i0, i0 -= kBS) {
    const int nb = (int)(i1 - i0);
    const int64_t rows = i0 > kBS ? i0 - kBS : 0;  // rows above the next block
    const int blocks = 1 + (int)std::min<int64_t>((rows + 3) / 4, 1024);
    hipLaunchKernelGGL(backsub_step_kernel<T>, dim3(blocks), dim3(256), 0, s, U, ldu, yw, x,
                       (int)i0, nb, unit);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

}  // namespace

int backsub_f64(const double* U, int64_t ldu, const double* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s) {
  return backsub_impl<double>(U, ldu, y, incy, x, bnorm, n, unit, yw, s);
}

int backsub_f32(const float* U, int64_t ldu, const float* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s) {
  return backsub_impl<float>(U, ldu, y, incy, x, bnorm, n, unit, yw, s);
}

}  // namespace gelim

extern "C" int gelim_gpu_backsub(const double* dU, int64_t ldu, const double* dy, int64_t incy,
                                 double* dx, double* dbnorm, int64_t n, int unit, void* stream) {
  if (n <= 0) return GELIM_FAIL(GELIM_E_ARG, "backsub: n <= 0");
  hipStream_t s = (hipStream_t)stream;
  double* yw = nullptr;
  HIP_TRY(hipMallocAsync((void**)&yw, sizeof(double) * n, s));
  int rc = gelim::backsub_f64(dU, ldu, dy, incy, dx, dbnorm, n, unit, yw, s);
  HIP_TRY(hipFreeAsync(yw, s));
  return rc;
}
