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
//                      stages its 64 multipliers in LDS and keeps its pivot-
//                      row element in a register (the register-resident form
//                      of "pivot row in LDS": every lane reuses it 64 times).
// Templated on T (double = reference precision; float = the north-star fp32
// path, exact on the synthetic internal matrix).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kPivThreads = 1024;
constexpr int kElimCols = 256;
constexpr int kElimRows = 64;

template <typename T>
__global__ __launch_bounds__(kPivThreads) void pivot_kernel(T* __restrict__ A, int64_t lda, int n,
                                                            int i, int mode, T* __restrict__ mcol,
                                                            int* __restrict__ info) {
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
  if (piv == T(0)) return;  // singular: info already set

  // pass 2: swap rows i <-> p over columns i..n (n = b) and scale row i
  T* ri = A + (int64_t)i * lda;
  T* rp = A + (int64_t)p * lda;
  const bool scale = piv != T(1);
  for (int c = i + t; c <= n; c += kPivThreads) {
    const T vi = ri[c];
    const T vp = (p != i) ? rp[c] : vi;
    if (p != i) rp[c] = vi;
    T nv = vp;
    if (scale) nv = (c == i) ? T(1) : vp / piv;
    ri[c] = nv;
  }
  if (t == 0 && p != i) mcol[p] = s_aii;  // multiplier of the row that moved to p
}

template <typename T>
__global__ __launch_bounds__(kElimCols) void eliminate_kernel(T* __restrict__ A, int64_t lda,
                                                              int n, int i,
                                                              const T* __restrict__ mcol) {
  __shared__ T s_m[kElimRows];
  const int t = threadIdx.x;
  const int r0 = i + 1 + blockIdx.y * kElimRows;
  if (t < kElimRows) s_m[t] = (r0 + t < n) ? mcol[r0 + t] : T(0);
  __syncthreads();
  const int c = i + blockIdx.x * kElimCols + t;
  if (c > n) return;
  const T u = A[(int64_t)i * lda + c];  // pivot-row element, reused kElimRows times
  const int rows = min(kElimRows, n - r0);
  T* a = A + (int64_t)r0 * lda + c;
  if (c == i) {
    for (int rr = 0; rr < rows; ++rr) a[(int64_t)rr * lda] = T(0);
  } else {
#pragma unroll 8
    for (int rr = 0; rr < rows; ++rr) a[(int64_t)rr * lda] -= s_m[rr] * u;
  }
}

}  // namespace

template <typename T>
int pivot_elimination(T* A, int64_t lda, int64_t n, int mode, T* mcol, int* info,
                      hipStream_t s) {
  for (int64_t i = 0; i < n; ++i) {
    hipLaunchKernelGGL(pivot_kernel<T>, dim3(1), dim3(kPivThreads), 0, s, A, lda, (int)n, (int)i,
                       mode, mcol, info);
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

template int pivot_elimination<double>(double*, int64_t, int64_t, int, double*, int*,
                                       hipStream_t);
template int pivot_elimination<float>(float*, int64_t, int64_t, int, float*, int*, hipStream_t);

}  // namespace gelim
