// Distributed randomised solver (parallel/dist_rbt.py, GaussSolver's
// "hip-rbt" over RCCL): the kernels that are specific to a rank's slice of
// the system.  The factorisation itself reuses the single-GPU pieces
// (lu_mixed.hip Gauss-Jordan block inverse, dgemm.hip fp64 MFMA GEMM).
//
// Layout (one process per GPU): 128-column blocks, block g on rank g % P, a
// rank's blocks stored left to right.  The order is padded to np, a multiple
// of 512 P, so that h / 128 = np / 512 blocks is a multiple of P: a butterfly
// column group {j, j + h, j + 2h, j + 3h} then lies on ONE rank, at local
// columns {jl, jl + hl, jl + 2hl, jl + 3hl} (hl = nloc / 4), and the
// transform M = U^T A V needs no communication -- U mixes rows, which every
// rank holds in full.
//
// Reference: the MPI program keeps every worker busy at every pivot step
// (OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:130-199); here every rank
// updates its own columns with every broadcast block, and there is no
// per-column collective at all (no pivot search).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <string>

#include "device_common.h"
#include "gelim/internal.h"
#include "rbt.h"

namespace gelim {
int dgemm_capped(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate);

namespace {

constexpr int NB = 128;  // block = the single-GPU engine's (lu_mixed.hip)

// M_loc = (U^T A V) restricted to this rank's columns.  Thread (i, jl): row
// group i (rows i + q h), local column group jl (local columns jl + p hl),
// whose global group index is j = (jl / 128 * P + r) * 128 + jl % 128.
// mbs > 0: M is column-block-major -- local block c (columns 128 c ..) is the
// slab at M + c * mbs, rows at ldm (= 128) inside it.
__global__ __launch_bounds__(256) void drbt_transform_kernel(const double* __restrict__ A, int64_t lda,
                                                             double* __restrict__ M, int64_t ldm, int64_t mbs, int np,
                                                             int nloc, int P, int r, const double* __restrict__ ud,
                                                             const double* __restrict__ vd) {
  const int h = np / 4, hl = nloc / 4;
  const int jl = blockIdx.x * 256 + threadIdx.x;
  const int i = blockIdx.y;
  if (jl >= hl) return;
  const int j = ((jl / NB) * P + r) * NB + jl % NB;
  double a[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) a[q][p] = A[(int64_t)(i + q * h) * lda + jl + p * hl];
  double U[4][4], V[4][4];
  rbt::group_w(ud, h, i, U);
  rbt::group_w(vd, h, j, V);
  double t[4][4];  // U^T a
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      double v = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) v += U[c][q] * a[c][p];
      t[q][p] = v;
    }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      double v = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) v += t[q][c] * V[c][p];
      const int col = jl + p * hl;
      const int64_t at = mbs ? (col / NB) * mbs + (int64_t)(i + q * h) * ldm + col % NB
                             : (int64_t)(i + q * h) * ldm + col;
      M[at] = v;
    }
}

// One super-block of the distributed block-triangular solves (S = nbs * 128
// equations, every rank redundantly): Fs (S x S, lds) is the gathered
// super-diagonal block of the factor, Dinv (nbs x 128 x 128) the inverses of
// its diagonal blocks, rhs the right-hand side already reduced over ranks.
//   lower: y_b = rhs_b - sum_{j<b} F_bj x_j,  x_b = Dinv_b y_b  (b ascending; y saved)
//   upper: t_b = rhs_b - sum_{j>b} F_bj x_j,  x_b = Dinv_b t_b  (b descending)
// 16 waves; wave w owns rows 8w .. 8w+7 of the current block, lanes stride
// the columns (coalesced row reads), one wave sum per row.
constexpr int kSsThreads = 1024;

__global__ __launch_bounds__(kSsThreads) void super_solve_kernel(const double* __restrict__ Fs, int64_t lds,
                                                                 const double* __restrict__ Dinv, int nbs,
                                                                 const double* __restrict__ rhs,
                                                                 double* __restrict__ x, double* __restrict__ ysave,
                                                                 int upper) {
  extern __shared__ double xs[];  // S solved values, then 128 of scratch
  double* yb = xs + nbs * NB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kRows = NB / (kSsThreads / 64);  // 8 rows per wave
  for (int s = 0; s < nbs; ++s) {
    const int b = upper ? nbs - 1 - s : s;
    // already-solved columns: [0, 128 b) (lower) or [128 (b+1), S) (upper)
    const int c0 = upper ? NB * (b + 1) : 0, c1 = upper ? NB * nbs : NB * b;
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int row = NB * b + kRows * wave + k;
      double acc = 0.0;
      for (int c = c0 + lane; c < c1; c += 64) acc = fma(Fs[(int64_t)row * lds + c], xs[c], acc);
      acc = dev::wave_sum(acc);
      if (lane == 0) {
        const double y = rhs[row] - acc;
        yb[row - NB * b] = y;
        if (ysave) ysave[row] = y;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int rr = kRows * wave + k;
      const double* d = Dinv + ((int64_t)b * NB + rr) * NB;
      double acc = fma(d[lane], yb[lane], 0.0);
      acc = fma(d[lane + 64], yb[lane + 64], acc);
      acc = dev::wave_sum(acc);
      if (lane == 0) {
        xs[NB * b + rr] = acc;
        x[NB * b + rr] = acc;
      }
    }
    __syncthreads();
  }
}

// y[i] += alpha * sum_c A[i][c] x[c] for i < m (c < k): one wave per row.
__global__ __launch_bounds__(256) void gemv_acc_kernel(const double* __restrict__ A, int64_t lda, int m, int k,
                                                       const double* __restrict__ x, double* __restrict__ y,
                                                       double alpha) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  const double* a = A + (int64_t)row * lda;
  double acc = 0.0;
  for (int c = lane; c < k; c += 64) acc = fma(a[c], x[c], acc);
  acc = dev::wave_sum(acc);
  if (lane == 0) y[row] += alpha * acc;
}

// y[i] = sum_c A[i][c] x[c], w[i] = sum_c |A[i][c]| |x[c]| (a rank's share of
// the residual and of the componentwise backward error's denominator).
__global__ __launch_bounds__(256) void matvec_abs_kernel(const double* __restrict__ A, int64_t lda, int m, int k,
                                                         const double* __restrict__ x, double* __restrict__ y,
                                                         double* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= m) return;
  const double* a = A + (int64_t)row * lda;
  double acc = 0.0, aw = 0.0;
  for (int c = lane; c < k; c += 64) {
    const double av = a[c], xv = x[c];
    acc = fma(av, xv, acc);
    aw = fma(fabs(av), fabs(xv), aw);
  }
  acc = dev::wave_sum(acc);
  aw = dev::wave_sum(aw);
  if (lane == 0) {
    y[row] = acc;
    w[row] = aw;
  }
}

}  // namespace
}  // namespace gelim

// M (np x nloc, ldm) = this rank's columns of U^T A V, A (np x nloc, lda) the
// rank's columns of the padded system.  np a multiple of 512 P, nloc = np / P.
// mbs > 0: M column-block-major (128-column slabs mbs doubles apart, ldm = 128).
extern "C" int gelim_drbt_transform(const double* A, int64_t lda, double* M, int64_t ldm, int64_t mbs, int64_t np,
                                    int64_t nloc, int P, int r, const double* ud, const double* vd, void* stream) {
  if (!A || !M || !ud || !vd || P < 1 || r < 0 || r >= P || np % (512 * (int64_t)P) || nloc * P != np ||
      lda < nloc || (mbs ? (ldm != gelim::NB || mbs < np * ldm) : ldm < nloc) || np > INT32_MAX)
    return GELIM_FAIL(GELIM_E_ARG, "drbt_transform: bad layout (np must be a multiple of 512 P, nloc = np / P)");
  const int64_t h = np / 4, hl = nloc / 4;
  if (h > 65535) return GELIM_FAIL(GELIM_E_ARG, "drbt_transform: order too large for the grid");
  const dim3 grid((unsigned)((hl + 255) / 256), (unsigned)h);
  hipLaunchKernelGGL(gelim::drbt_transform_kernel, grid, dim3(256), 0, (hipStream_t)stream, A, lda, M, ldm, mbs,
                     (int)np, (int)nloc, P, r, ud, vd);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// One super-block solve (see super_solve_kernel): S = nbs * 128 <= 8192.
extern "C" int gelim_drbt_super_solve(const double* Fs, int64_t lds, const double* Dinv, int nbs, const double* rhs,
                                      double* x, double* ysave, int upper, void* stream) {
  if (!Fs || !Dinv || !rhs || !x || nbs < 1 || nbs > 64 || lds < (int64_t)nbs * gelim::NB)
    return GELIM_FAIL(GELIM_E_ARG, "drbt_super_solve: bad argument");
  const size_t lds_bytes = sizeof(double) * ((size_t)nbs * gelim::NB + gelim::NB);
  hipLaunchKernelGGL(gelim::super_solve_kernel, dim3(1), dim3(gelim::kSsThreads), lds_bytes, (hipStream_t)stream, Fs,
                     lds, Dinv, nbs, rhs, x, ysave, upper);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// y[:m] += alpha A x (A m x k, lda).
extern "C" int gelim_drbt_gemv(const double* A, int64_t lda, int64_t m, int64_t k, const double* x, double* y,
                               double alpha, void* stream) {
  if (m <= 0 || k <= 0) return GELIM_OK;
  if (!A || !x || !y || lda < k || m > INT32_MAX || k > INT32_MAX) return GELIM_FAIL(GELIM_E_ARG, "drbt_gemv");
  hipLaunchKernelGGL(gelim::gemv_acc_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, A, lda,
                     (int)m, (int)k, x, y, alpha);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// y = A x, w = |A| |x| (A m x k, lda).
extern "C" int gelim_drbt_matvec_abs(const double* A, int64_t lda, int64_t m, int64_t k, const double* x, double* y,
                                     double* w, void* stream) {
  if (m <= 0) return GELIM_OK;
  if (!A || !x || !y || !w || lda < k || m > INT32_MAX || k > INT32_MAX)
    return GELIM_FAIL(GELIM_E_ARG, "drbt_matvec_abs");
  hipLaunchKernelGGL(gelim::matvec_abs_kernel, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, A,
                     lda, (int)m, (int)k, x, y, w);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// C = alpha A B (accumulate = 0) or C += alpha A B, on at most max_wg CUs
// (0: uncapped) -- the fp64 MFMA GEMM of dgemm.hip with the accumulate switch.
extern "C" int gelim_gpu_dgemm_ex(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb,
                                  int64_t M, int64_t N, int64_t K, double alpha, int accumulate, int max_wg,
                                  void* stream) {
  return gelim::dgemm_capped(C, ldc, A, lda, B, ldb, M, N, K, alpha, max_wg, (hipStream_t)stream, accumulate);
}
