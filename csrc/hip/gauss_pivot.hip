// The reference's per-pivot Gaussian elimination, on the GPU.
//
// Same algorithm and the same arithmetic per element as the CPU reference
// (forward elimination to a UNIT upper triangle, pivot row divided by the
// pivot, b carried as the augmented column n):
//   getPivot + row scaling  (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:123-169,
//                            Pthreads/Version-1/gauss_internal_input.c:75-121)
//   elimination             (gauss_external_input.c:172-180)
// The reference's five CPU strategies (fork-join, column-blocked,
// persistent+barrier, OpenMP, MPI scatter/gather) all collapse into the same
// two kernels per pivot on one HIP stream (captured into a hipGraph by the
// plan):
//   pivot_kernel     : ONE 1024-thread workgroup — arg-max over the column,
//                      row swap, pivot-row scaling, and it snapshots the
//                      multiplier column into a side vector so the
//                      elimination grid never races on A[j][i];
//   eliminate_kernel : 2-D grid over the trailing block, each workgroup
//                      stages its 16 multipliers in LDS and keeps its pivot-
//                      row element in a register (the register-resident form
//                      of "pivot row in LDS": every lane reuses it 16 times),
//                      all 16 loads of a lane in flight at once.
// Templated on T (double = reference precision; float = the north-star fp32
// path, exact on the synthetic internal matrix).
//
// The factors are kept (LAPACK style), so a plan can re-solve a new right-
// hand side in O(n^2) (pivot_resolve, used by mixed-precision refinement):
// rows are swapped over their FULL width, the eliminated entries hold the
// multipliers m_r (the column's value before the step), ipiv[i] the pivot
// row and diag[i] the pivot value.  With the pivot row scaled to a unit
// diagonal, A = P^T L~ U~ where L~ = (multipliers, diag on the diagonal) and
// U~ = the unit upper triangle left in A.
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kPivThreads = 1024;
constexpr int kElimCols = 256;
constexpr int kElimRows = 16;

template <typename T>
__global__ __launch_bounds__(kPivThreads) void pivot_kernel(T* __restrict__ A, int64_t lda, int n,
                                                            int i, int mode, T* __restrict__ mcol,
                                                            int* __restrict__ info, int* __restrict__ ipiv,
                                                            double* __restrict__ diag) {
  __shared__ double s_val[16];
  __shared__ int s_idx[16];
  __shared__ int s_p;
  __shared__ T s_piv, s_aii;
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;

  // pass 1: snapshot the column (multipliers) and find the pivot row
  double best = -1.0;
  int bidx = INT_MAX;
  for (int r = i + t; r < n; r += kPivThreads) {
    const T v = A[(int64_t)r * lda + i];
    mcol[r] = v;
    const double key = dev::pivot_key(v, r == i, mode);
    if (key > best) {
      best = key;
      bidx = r;
    }
  }
  dev::wave_argmax(best, bidx);
  if (lane == 0) {
    s_val[wave] = best;
    s_idx[wave] = bidx;
  }
  __syncthreads();
  if (wave == 0) {
    double v = lane < 16 ? s_val[lane] : -1.0;
    int id = lane < 16 ? s_idx[lane] : INT_MAX;
    dev::group_argmax(v, id, 16);
    if (lane == 0) {
      s_p = id;
      if (v <= 0.0) {
        if (*info == 0) *info = i + 1;
        s_p = i;
      }
      s_piv = A[(int64_t)s_p * lda + i];
      s_aii = A[(int64_t)i * lda + i];
    }
  }
  __syncthreads();
  const int p = s_p;
  const T piv = s_piv;
  if (t == 0) {
    ipiv[i] = p;
    diag[i] = (double)piv;
  }
  // singular: info is set; the column is all zeros, so the elimination
  // kernel of this step (which checks the scaled diagonal) does nothing
  if (piv == T(0)) return;

  // pass 2: swap rows i <-> p over the full width (the stored multipliers
  // left of column i move with their rows) and scale row i from column i on
  T* ri = A + (int64_t)i * lda;
  T* rp = A + (int64_t)p * lda;
  const bool scale = piv != T(1);
  for (int c = t; c <= n; c += kPivThreads) {
    if (c < i && p == i) continue;
    const T vi = ri[c];
    const T vp = (p != i) ? rp[c] : vi;
    if (p != i) rp[c] = vi;
    T nv = vp;
    if (scale && c >= i) nv = (c == i) ? T(1) : vp / piv;
    ri[c] = nv;
  }
  if (t == 0 && p != i) mcol[p] = s_aii;  // multiplier of the row that moved to p
}

template <typename T>
__global__ __launch_bounds__(kElimCols) void eliminate_kernel(T* __restrict__ A, int64_t lda,
                                                              int n, int i,
                                                              const T* __restrict__ mcol) {
  // 256 columns x kElimRows rows per workgroup, one column per thread: the
  // pivot-row element u stays in a register, the rows' multipliers come from
  // LDS, and all kElimRows loads of a thread are issued before any FMA (one
  // memory round trip per step instead of one per 8 rows: the step is a
  // bandwidth/latency-bound rank-1 update, ~(n-i)^2 x 2 x sizeof(T) bytes;
  // 2048^2 fp64: 53.7 -> 27.7 ms per solve with 64-row workgroups before)
  __shared__ T s_m[kElimRows];
  const int t = threadIdx.x;
  const int r0 = i + 1 + blockIdx.y * kElimRows;
  if (t < kElimRows) s_m[t] = (r0 + t < n) ? mcol[r0 + t] : T(0);
  __syncthreads();
  const int c = i + blockIdx.x * kElimCols + t;
  if (c > n) return;
  // a zero pivot left row i unscaled (its diagonal is 0, not 1): skip the step
  if (A[(int64_t)i * lda + i] == T(0)) return;
  const T u = A[(int64_t)i * lda + c];  // pivot-row element, reused kElimRows times
  const int rows = min(kElimRows, n - r0);
  T* a = A + (int64_t)r0 * lda + c;
  if (c == i) {
    // the eliminated column keeps the multipliers (L~ of the stored factors)
    for (int rr = 0; rr < rows; ++rr) a[(int64_t)rr * lda] = s_m[rr];
    return;
  }
  T v[kElimRows];
#pragma unroll
  for (int rr = 0; rr < kElimRows; ++rr) v[rr] = a[(int64_t)min(rr, rows - 1) * lda];  // clamped: no branches
#pragma unroll
  for (int rr = 0; rr < kElimRows; ++rr)
    if (rr < rows) a[(int64_t)rr * lda] = v[rr] - s_m[rr] * u;
}

}  // namespace

// Re-solve with the stored factors: y = L~^-1 P c (one workgroup: blocks of
// 64 rows, wave 0 solves the diagonal triangle, all waves update the rows
// below; y lives in LDS), accumulated in fp64 from T-precision factors.
// The row permutation is rebuilt from ipiv by lane 0 first (n serial swaps
// in LDS).  The unit upper solve that follows is backsub.hip's.
template <typename T>
__global__ __launch_bounds__(1024) void lower_resolve_kernel(const T* __restrict__ A, int64_t lda, int n,
                                                             const int* __restrict__ ipiv,
                                                             const double* __restrict__ diag,
                                                             const double* __restrict__ c, T* __restrict__ y) {
  extern __shared__ double ys[];              // [n] values, then [n] int permutation
  int* perm = reinterpret_cast<int*>(ys + n);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int i = t; i < n; i += 1024) perm[i] = i;
  __syncthreads();
  if (t == 0)
    for (int i = 0; i < n; ++i) {
      const int p = ipiv[i];
      const int a = perm[i];
      perm[i] = perm[p];
      perm[p] = a;
    }
  __syncthreads();
  for (int i = t; i < n; i += 1024) ys[i] = c[perm[i]];
  __syncthreads();
  for (int b0 = 0; b0 < n; b0 += 64) {
    const int nb = min(64, n - b0);
    if (wave == 0) {
      // lane l owns row b0 + l of the block; serial over the block columns
      double v = lane < nb ? ys[b0 + lane] : 0.0;
      for (int j = 0; j < nb; ++j) {
        const double xj_l = v / diag[b0 + j];
        const double xj = __shfl(xj_l, j);
        if (lane == j) v = xj;
        if (lane > j && lane < nb) v = fma(-(double)A[(int64_t)(b0 + lane) * lda + b0 + j], xj, v);
      }
      if (lane < nb) ys[b0 + lane] = v;
    }
    __syncthreads();
    // rows below the block: one wave per row, lanes over the block columns
    for (int r = b0 + nb + wave; r < n; r += 16) {
      double acc = lane < nb ? (double)A[(int64_t)r * lda + b0 + lane] * ys[b0 + lane] : 0.0;
      acc = dev::wave_sum(acc);
      if (lane == 0) ys[r] -= acc;
    }
    __syncthreads();
  }
  for (int i = t; i < n; i += 1024) y[i] = (T)ys[i];
}

template <typename T>
int pivot_lower_resolve(const T* A, int64_t lda, int64_t n, const int* ipiv, const double* diag, const double* c,
                        T* y, hipStream_t s) {
  const size_t lds = (size_t)n * (sizeof(double) + sizeof(int));
  if (lds > 160 * 1024) return GELIM_FAIL(GELIM_E_ARG, "resolve: n too large for the one-workgroup solve");
  // more than 64 KiB of dynamic LDS (n > ~5460) must be requested explicitly
  static const bool attr = hipFuncSetAttribute((const void*)lower_resolve_kernel<T>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  if (!attr && lds > 64 * 1024) return GELIM_FAIL(GELIM_E_HIP, "resolve: LDS attribute refused");
  hipLaunchKernelGGL(lower_resolve_kernel<T>, dim3(1), dim3(1024), lds, s, A, lda, (int)n, ipiv, diag, c, y);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

template int pivot_lower_resolve<double>(const double*, int64_t, int64_t, const int*, const double*, const double*,
                                         double*, hipStream_t);
template int pivot_lower_resolve<float>(const float*, int64_t, int64_t, const int*, const double*, const double*,
                                        float*, hipStream_t);

template <typename T>
int pivot_elimination(T* A, int64_t lda, int64_t n, int mode, T* mcol, int* info, hipStream_t s, int* ipiv,
                      double* diag) {
  for (int64_t i = 0; i < n; ++i) {
    hipLaunchKernelGGL(pivot_kernel<T>, dim3(1), dim3(kPivThreads), 0, s, A, lda, (int)n, (int)i,
                       mode, mcol, info, ipiv, diag);
    HIP_TRY(hipGetLastError());
    const int64_t rows = n - 1 - i;
    if (rows <= 0) continue;
    dim3 grid((unsigned)((n + 1 - i + kElimCols - 1) / kElimCols),
              (unsigned)((rows + kElimRows - 1) / kElimRows));
    hipLaunchKernelGGL(eliminate_kernel<T>, grid, dim3(kElimCols), 0, s, A, lda, (int)n, (int)i,
                       (const T*)mcol);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

template int pivot_elimination<double>(double*, int64_t, int64_t, int, double*, int*, hipStream_t, int*, double*);
template int pivot_elimination<float>(float*, int64_t, int64_t, int, float*, int*, hipStream_t, int*, double*);

}  // namespace gelim
