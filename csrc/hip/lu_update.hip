// Trailing-matrix update of the blocked LU:
//   swap_trsm : apply the panel's w row interchanges to the columns right of
//               the panel, then U12 = L11^{-1} A12 (unit lower triangle);
//   gemm      : A22 -= L21 * U12 on the fp64 matrix cores
//               (v_mfma_f64_16x16x4_f64).
// Together they are the blocked form of the reference's O(n^3) hot loop
// `matrix[j][k] -= pivotval * matrix[i][k]`
// (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:172-180): w rank-1
// updates fused into one rank-w GEMM so the elimination runs on MFMA instead
// of streaming the trailing matrix through memory once per pivot.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kSwapThreads = 256;
constexpr int kMaxPairs = 64;  // 2 * max panel width

// Net row permutation of w sequential interchanges (j <-> piv[j], piv[j] >= j)
// as (dst, src) pairs: new_row[dst] = old_row[src].  Computed by wave 0:
// lanes find first occurrences in parallel, lane 0 runs the O(w) simulation.
__device__ int build_pairs(const int* __restrict__ piv, int w, int* s_dst, int* s_src,
                           int* s_slot, int* s_pos, int* s_low) {
  const int t = threadIdx.x;
  if (t < w) {
    const int pj = piv[t];
    int slot = -1;
    if (pj >= w) {
      for (int q = 0; q <= t; ++q)
        if (piv[q] == pj) {
          slot = q;
          break;
        }
    }
    s_slot[t] = slot;
    s_pos[t] = t;
    s_low[t] = pj;
  }
  __syncthreads();
  __shared__ int s_np;
  if (t == 0) {
    for (int j = 0; j < w; ++j) {
      const int pj = piv[j];
      if (pj == j) continue;
      if (pj < w) {
        int x = s_pos[j];
        s_pos[j] = s_pos[pj];
        s_pos[pj] = x;
      } else {
        const int sl = s_slot[j];
        int x = s_pos[j];
        s_pos[j] = s_low[sl];
        s_low[sl] = x;
      }
    }
    int np = 0;
    for (int r = 0; r < w; ++r)
      if (s_pos[r] != r) {
        s_dst[np] = r;
        s_src[np] = s_pos[r];
        ++np;
      }
    for (int j = 0; j < w; ++j)
      if (s_slot[j] == j && s_low[j] != piv[j]) {
        s_dst[np] = piv[j];
        s_src[np] = s_low[j];
        ++np;
      }
    s_np = np;
  }
  __syncthreads();
  return s_np;
}

template <int W>
__global__ __launch_bounds__(kSwapThreads) void swap_trsm_kernel(
    double* __restrict__ C, int64_t ldc, int ncols, const double* __restrict__ L, int64_t ldl,
    int w, const int* __restrict__ piv, double* __restrict__ tmp) {
  __shared__ double s_L[W][W];
  __shared__ int s_dst[kMaxPairs], s_src[kMaxPairs], s_slot[W], s_pos[W], s_low[W];
  const int t = threadIdx.x;
  for (int e = t; e < w * w; e += kSwapThreads) {
    const int r = e / w, c = e % w;
    s_L[r][c] = (c < r) ? L[(int64_t)r * ldl + c] : 0.0;
  }
  const int np = build_pairs(piv, w, s_dst, s_src, s_slot, s_pos, s_low);

  const int64_t c = (int64_t)blockIdx.x * kSwapThreads + t;
  if (c >= ncols) return;
  double* col = C + c;
  // gather through a per-column scratch (tmp[e*ncols + c]) so every source is
  // read before any destination is written
  if (np > 0) {
    for (int e = 0; e < np; ++e) tmp[(int64_t)e * ncols + c] = col[(int64_t)s_src[e] * ldc];
    for (int e = 0; e < np; ++e) col[(int64_t)s_dst[e] * ldc] = tmp[(int64_t)e * ncols + c];
  }
  double x[W];
  const double* pl = col;
#pragma unroll
  for (int j = 0; j < W; ++j, pl += ldc) x[j] = (j < w) ? *pl : 0.0;
  // column-oriented forward substitution: x[i] is final at step i and is
  // stored right away; the scheduling fence per step keeps the compiler from
  // hoisting all W^2/2 LDS reads of L11 into registers
  double* ps = col + ldc;
#pragma unroll
  for (int i = 0; i < W - 1; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const double xi = x[i];
#pragma unroll
    for (int j = i + 1; j < W; ++j) x[j] -= s_L[j][i] * xi;
    if (i + 1 < w) *ps = x[i + 1];
    ps += ldc;
  }
}

// Pair-list form used by the solver plan: the panel kernel already emitted
// the net row movement (pairs[0] = count, then (dst, src) per pair), so there
// is no per-block reconstruction.  Per column (one thread): every touched
// source row is loaded before anything is stored, the top w rows are staged
// in this thread's LDS column for the triangular solve, other destinations
// are written straight back.
template <int W>
__global__ __launch_bounds__(kSwapThreads) void pairs_trsm_kernel(
    double* __restrict__ C, int64_t ldc, int ncols, const double* __restrict__ L, int64_t ldl,
    int w, const int* __restrict__ pairs) {
  __shared__ double s_L[W][W];
  __shared__ double xs[W][kSwapThreads];
  __shared__ int s_pair[1 + 4 * W];
  const int t = threadIdx.x;
  for (int e = t; e < W * W; e += kSwapThreads) {
    const int r = e / W, c = e % W;
    s_L[r][c] = (c < r && r < w) ? L[(int64_t)r * ldl + c] : 0.0;
  }
  if (t < 1 + 4 * W) s_pair[t] = (t == 0 || t <= 2 * pairs[0]) ? pairs[t] : 0;
  __syncthreads();
  const int np = s_pair[0];
  const int64_t c = (int64_t)blockIdx.x * kSwapThreads + t;
  if (c >= ncols) return;
  double* col = C + c;
  double g[2 * W];
#pragma unroll
  for (int e = 0; e < 2 * W; ++e)
    g[e] = (e < np) ? col[(int64_t)s_pair[2 + 2 * e] * ldc] : 0.0;
  const double* pl = col;
#pragma unroll
  for (int j = 0; j < W; ++j, pl += ldc) xs[j][t] = (j < w) ? *pl : 0.0;
#pragma unroll
  for (int e = 0; e < 2 * W; ++e) {
    if (e < np) {
      const int d = s_pair[1 + 2 * e];
      if (d < w) xs[d][t] = g[e];
      else col[(int64_t)d * ldc] = g[e];
    }
  }
  double x[W];
#pragma unroll
  for (int j = 0; j < W; ++j) x[j] = xs[j][t];
  double* ps = col;
#pragma unroll
  for (int i = 0; i < W; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const double xi = x[i];
    if (i < w) *ps = xi;  // final U12 row i
    ps += ldc;
#pragma unroll
    for (int j = i + 1; j < W; ++j) x[j] -= s_L[j][i] * xi;
  }
}

// ---- fp64 MFMA GEMM: C -= L * U --------------------------------------------
// Workgroup tile 64x64, 4 waves as 2x2, each wave 32x32 = 2x2 blocks of the
// 16x16x4 f64 MFMA.  Operand maps (gfx950, f64): A lane l holds
// A[l&15][k=l>>4], B lane l holds B[k=l>>4][l&15]; C/D register r of lane l is
// C[row=(l>>4)+4r][col=l&15]  (cdna_hip_programming.md §3: f64 does NOT use
// the f32 C/D map).
constexpr int kGemmThreads = 256;

__global__ __launch_bounds__(kGemmThreads) void gemm_update_f64_kernel(
    double* __restrict__ C, int64_t ldc, const double* __restrict__ L, int64_t ldl,
    const double* __restrict__ U, int64_t ldu, int M, int N, int K) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int m0 = blockIdx.y * 64 + (wave >> 1) * 32;
  const int n0 = blockIdx.x * 64 + (wave & 1) * 32;

  dev::d4 acc[2][2];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = n0 + nb * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + mb * 16 + q + 4 * r;
        acc[mb][nb][r] = (row < M && col < N) ? C[(int64_t)row * ldc + col] : 0.0;
      }
    }

  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + q;
    double a[2], b[2];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int row = m0 + mb * 16 + r16;
      a[mb] = (row < M && k < K) ? -L[(int64_t)row * ldl + k] : 0.0;
    }
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = n0 + nb * 16 + r16;
      b[nb] = (col < N && k < K) ? U[(int64_t)k * ldu + col] : 0.0;
    }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mb], b[nb], acc[mb][nb], 0, 0, 0);
  }

#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int col = n0 + nb * 16 + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + mb * 16 + q + 4 * r;
        if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[mb][nb][r];
      }
    }
}

template <int W>
int launch_swap_trsm(double* C, int64_t ldc, int64_t ncols, const double* L, int64_t ldl,
                     int64_t w, const int* piv, double* tmp, hipStream_t s) {
  const int blocks = (int)((ncols + kSwapThreads - 1) / kSwapThreads);
  hipLaunchKernelGGL((swap_trsm_kernel<W>), dim3(blocks), dim3(kSwapThreads), 0, s, C, ldc,
                     (int)ncols, L, ldl, (int)w, piv, tmp);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// tmp must hold 2*w*ncols doubles.
int swap_trsm(double* C, int64_t ldc, int64_t ncols, const double* L, int64_t ldl, int64_t w,
              const int* piv, double* tmp, hipStream_t s) {
  if (ncols <= 0) return GELIM_OK;
  if (w <= 2) return launch_swap_trsm<2>(C, ldc, ncols, L, ldl, w, piv, tmp, s);
  if (w <= 4) return launch_swap_trsm<4>(C, ldc, ncols, L, ldl, w, piv, tmp, s);
  if (w <= 8) return launch_swap_trsm<8>(C, ldc, ncols, L, ldl, w, piv, tmp, s);
  if (w <= 16) return launch_swap_trsm<16>(C, ldc, ncols, L, ldl, w, piv, tmp, s);
  if (w <= 32) return launch_swap_trsm<32>(C, ldc, ncols, L, ldl, w, piv, tmp, s);
  return GELIM_FAIL(GELIM_E_ARG, "swap_trsm: w > 32");
}

int pairs_trsm(double* C, int64_t ldc, int64_t ncols, const double* L, int64_t ldl, int64_t w,
               const int* pairs, hipStream_t s) {
  if (ncols <= 0) return GELIM_OK;
  const int blocks = (int)((ncols + kSwapThreads - 1) / kSwapThreads);
#define GELIM_PT(WW)                                                                        \
  hipLaunchKernelGGL((pairs_trsm_kernel<WW>), dim3(blocks), dim3(kSwapThreads), 0, s, C, ldc, \
                     (int)ncols, L, ldl, (int)w, pairs)
  if (w <= 2) GELIM_PT(2);
  else if (w <= 4) GELIM_PT(4);
  else if (w <= 8) GELIM_PT(8);
  else if (w <= 16) GELIM_PT(16);
  else return GELIM_FAIL(GELIM_E_ARG, "pairs_trsm: w > 16");
#undef GELIM_PT
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int dgemm(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
          int64_t N, int64_t K, double alpha, hipStream_t s);

int gemm_update(double* C, int64_t ldc, const double* L, int64_t ldl, const double* U,
                int64_t ldu, int64_t M, int64_t N, int64_t K, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return GELIM_OK;
  // the LDS-tiled MFMA GEMM (dgemm.hip) whenever its operand contract holds;
  // the register-only kernel below covers odd K / unaligned views
  if (!(K & 1) && !(ldl & 1) && !(ldu & 1) && !(((uintptr_t)L | (uintptr_t)U) & 15) && (!(N & 1) || ldu > N) &&
      ldl >= K && ldu >= N && ldc >= N)
    return dgemm(C, ldc, L, ldl, U, ldu, M, N, K, -1.0, s);
  dim3 grid((unsigned)((N + 63) / 64), (unsigned)((M + 63) / 64));
  hipLaunchKernelGGL(gemm_update_f64_kernel, grid, dim3(kGemmThreads), 0, s, C, ldc, L, ldl, U,
                     ldu, (int)M, (int)N, (int)K);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace gelim

extern "C" int gelim_gpu_swap_trsm(double* dC, int64_t ldc, int64_t ncols, const double* dL,
                                   int64_t ldl, int64_t w, const int32_t* dpiv, int64_t nrows,
                                   void* stream) {
  (void)nrows;
  if (ncols <= 0) return GELIM_OK;
  double* tmp = nullptr;
  HIP_TRY(hipMallocAsync((void**)&tmp, sizeof(double) * 2 * w * ncols, (hipStream_t)stream));
  int rc = gelim::swap_trsm(dC, ldc, ncols, dL, ldl, w, dpiv, tmp, (hipStream_t)stream);
  HIP_TRY(hipFreeAsync(tmp, (hipStream_t)stream));
  return rc;
}

extern "C" int gelim_gpu_gemm_update(double* dC, int64_t ldc, const double* dL, int64_t ldl,
                                     const double* dU, int64_t ldu, int64_t M, int64_t N,
                                     int64_t K, void* stream) {
  return gelim::gemm_update(dC, ldc, dL, ldl, dU, ldu, M, N, K, (hipStream_t)stream);
}
