// Mixed-precision solver (GaussSolver backend "hip-mixed"): a random
// butterfly transform (RBT) of the system, a NO-pivoting blocked LU of the
// transformed matrix in fp32 on the matrix cores, and fp64 iterative
// refinement against the original system (the loop is in
// models/gauss_solver.py; when it does not reach the fp64 error class the
// solver falls back to the fp64 partial-pivoting engine by itself).
//
// Why: every exact partial-pivoting engine here is bound by its pivot chain
// (one global arg-max per column: ~4 us per column on the wide-panel leaves
// at n = 8192, profiles/leaf_fused_vs_2hop.txt), so an fp32 copy of the same
// algorithm would be just as slow.  A two-sided recursive butterfly
// transform U^T A V (Parker 1995; Baboulin, Dongarra et al. 2013) makes
// pivoting unnecessary with probability close to one, and the factorisation
// is then panel-free in the latency sense: per 128-column block one
// workgroup factors the 128 x 128 diagonal block, two column-/row-parallel
// triangular solves produce U12 and L21, and one fp32 MFMA GEMM
// (gemm_f32.hip, alpha = -1) updates the trailing matrix.  fp64 refinement
// (residual in fp64 on the ORIGINAL system) restores the fp64 error class
// (SURVEY.md §4.3 requires it: fp32 elimination alone fails saylr4 /
// orsreg_1).  The reference has no refinement and no fp32 Gauss
// (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182 is fp64).
//
// Depth-2 recursive butterfly: W = L1 L0, L0 = B<n> = 1/sqrt2 [R S; R -S]
// on (i, i + n/2), L1 = diag(B<n/2>_a, B<n/2>_b) on (i, i + n/4) and
// (i + n/2, i + 3n/4); R, S diagonal with entries exp(r / 10), r uniform in
// [-1/2, 1/2].  Both levels act on the index groups {i, i + h, i + 2h,
// i + 3h} (h = n/4) as one 4 x 4 matrix W_i, so M = U^T A V is ONE pass over
// A: every 4 x 4 group of entries becomes U_i^T A_g V_j (and fp32 on the way
// out).  The system is padded to np = a multiple of 128 with an identity
// block (b padded with zeros).
//
// Storage of the factors: L (unit lower, below the diagonal) and U (on and
// above it) overwrite the fp32 matrix, LAPACK style.  Solves: backsub.hip's
// persistent forward (unit lower) and back (upper) substitutions, fp64
// accumulation over the fp32 factors (np <= 16384: every 64-row block
// resident).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
int matmul_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N,
               int64_t K, int accumulate, int kernel, hipStream_t s, float alpha);
int backsub_f32(const float* U, int64_t ldu, const float* y, int64_t incy, double* x, double* bnorm, int64_t n,
                int unit, double* yw, hipStream_t s, const int* perm, int* err);
int fwdsub_unit_f32(const float* L, int64_t ldl, const double* y, float* out, int64_t n, double* xs,
                    unsigned* flags, hipStream_t s);

namespace {

constexpr int NB = 128;        // LU block
constexpr int kPadTo = NB;     // np multiple
constexpr int kLdsLd = NB + 1;  // diagonal-block LDS row stride (floats)

// ---- the butterfly group matrices -------------------------------------------
// d: 8 arrays of h doubles: R0[i], R0[i+h], S0[i], S0[i+h], Ra[i], Sa[i], Rb[i], Sb[i]
__device__ __forceinline__ void group_w(const double* __restrict__ d, int h, int i, double (&W)[4][4]) {
  const double r0 = d[i], r0h = d[h + i], s0 = d[2 * h + i], s0h = d[3 * h + i];
  const double ra = d[4 * h + i], sa = d[5 * h + i], rb = d[6 * h + i], sb = d[7 * h + i];
  // L0 (order i, i+h, i+2h, i+3h)
  const double L0[4][4] = {{r0, 0, s0, 0}, {0, r0h, 0, s0h}, {r0, 0, -s0, 0}, {0, r0h, 0, -s0h}};
  const double L1[4][4] = {{ra, sa, 0, 0}, {ra, -sa, 0, 0}, {0, 0, rb, sb}, {0, 0, rb, -sb}};
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      double v = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) v += L1[a][c] * L0[c][b];
      W[a][b] = 0.5 * v;  // (1/sqrt2)^2
    }
}

// M[g] = U_i^T A_g V_j for every 4 x 4 group; A is the n x n system (row
// major, lda), padded on the fly to np with an identity block.
__global__ __launch_bounds__(256) void rbt_matrix_kernel(const double* __restrict__ A, int64_t lda, int n, int np,
                                                        const double* __restrict__ ud, const double* __restrict__ vd,
                                                        float* __restrict__ M, int64_t ldm) {
  const int h = np / 4;
  const int j = blockIdx.x * 256 + threadIdx.x;  // column group
  const int i = blockIdx.y;                      // row group
  if (j >= h) return;
  double a[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int r = i + q * h, c = j + p * h;
      a[q][p] = (r < n && c < n) ? A[(int64_t)r * lda + c] : (r == c ? 1.0 : 0.0);
    }
  double U[4][4], V[4][4];
  group_w(ud, h, i, U);
  group_w(vd, h, j, V);
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
      M[(int64_t)(i + q * h) * ldm + j + p * h] = (float)v;
    }
}

// out = U^T [b; 0] (left) or out = V y (right), fp64 vectors of np entries
// (b: n entries with stride incb; the padding reads as 0)
__global__ __launch_bounds__(256) void rbt_vec_kernel(const double* __restrict__ b, int64_t incb, int n, int np,
                                                     const double* __restrict__ d, int transpose,
                                                     double* __restrict__ out) {
  const int h = np / 4;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= h) return;
  double W[4][4];
  group_w(d, h, i, W);
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = i + q * h;
    v[q] = r < n ? b[(int64_t)r * incb] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) s += (transpose ? W[c][q] : W[q][c]) * v[c];
    out[i + q * h] = s;
  }
}

// ---- blocked no-pivot LU ------------------------------------------------------
// One workgroup factors the NB x NB diagonal block at (k0, k0) in LDS: 8
// threads per row, one barrier per column.  info[0] = 1 + the first column
// whose pivot is zero or not finite (kept if set).
__global__ __launch_bounds__(1024) void diag_lu_kernel(float* __restrict__ A, int64_t lda, int k0,
                                                      int* __restrict__ info) {
  extern __shared__ float S[];  // [NB][kLdsLd]
  const int t = threadIdx.x, row = t >> 3, c8 = t & 7;
  float* Ar = A + (int64_t)(k0 + row) * lda + k0;
  for (int j = c8; j < NB; j += 8) S[row * kLdsLd + j] = Ar[j];
  __syncthreads();
  for (int k = 0; k < NB - 1; ++k) {
    if (row > k) {
      const float p = S[k * kLdsLd + k];
      const float l = S[row * kLdsLd + k] / p;
      // the row's 16 columns as one batch of independent LDS reads / FMAs /
      // writes (a static loop, predicated on j > k), not a dependent chain
      float v[NB / 8], u[NB / 8];
#pragma unroll
      for (int q = 0; q < NB / 8; ++q) {
        const int j = c8 + 8 * q;
        v[q] = S[row * kLdsLd + j];
        u[q] = S[k * kLdsLd + j];
      }
#pragma unroll
      for (int q = 0; q < NB / 8; ++q) {
        const int j = c8 + 8 * q;
        if (j > k) S[row * kLdsLd + j] = fmaf(-l, u[q], v[q]);
      }
      if (c8 == (k & 7)) S[row * kLdsLd + k] = l;
    }
    __syncthreads();
  }
  if (c8 == 0) {
    const float p = S[row * kLdsLd + row];
    if (!(p != 0.0f) || !isfinite(p)) atomicMin(info, k0 + row + 1);
  }
  for (int j = c8; j < NB; j += 8) Ar[j] = S[row * kLdsLd + j];
}

// Both off-diagonal triangular solves are lower-triangular solves on a
// 128 x 64 tile X held in LDS, one barrier per column k (row k of X is final
// once step k-1 is done and nobody writes it at step k):
//   U12 = L11^-1 A12        X = a 64-column slice of A12, L = L11 (unit);
//   L21 = A21 U11^-1  <=>  L21^T = U11^-T A21^T: X = a 64-row slice of A21,
//                           transposed, L = U11^T (its diagonal divisions
//                           deferred to the end: row k is not touched after
//                           its step).
// 256 threads: lane = column of X, wave = row group (rows i = rg mod 4).
constexpr int kXld = 65, kLld = NB + 1, kTile = 64;

template <bool UNIT>
__device__ __forceinline__ void tile_lower_solve(float* __restrict__ X, const float* __restrict__ L,
                                                 const float* __restrict__ rinv) {
  const int t = threadIdx.x, c = t & 63, rg = t >> 6;
  for (int k = 0; k < NB - 1; ++k) {
    const float xk = UNIT ? X[k * kXld + c] : X[k * kXld + c] * rinv[k];
    // this thread's 32 rows i = 4 q + rg as one batch (static loop, predicated
    // on i > k): independent LDS reads, FMAs and writes, pipelined
    float v[NB / 4], l[NB / 4];
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) {
      const int i = 4 * q + rg;
      v[q] = X[i * kXld + c];
      l[q] = L[i * kLld + k];
    }
#pragma unroll
    for (int q = 0; q < NB / 4; ++q) {
      const int i = 4 * q + rg;
      if (i > k) X[i * kXld + c] = fmaf(-l[q], xk, v[q]);
    }
    __syncthreads();
  }
  if (!UNIT)
    for (int i = rg; i < NB; i += 4) X[i * kXld + c] *= rinv[i];
  __syncthreads();
}

// U12 = L11^-1 A12 in place for columns [c0, c0 + ncols), 64 per workgroup.
__global__ __launch_bounds__(256) void trsm_u12_kernel(float* __restrict__ A, int64_t lda, int k0, int c0, int ncols) {
  extern __shared__ float lds[];
  float* L = lds;                // [NB][kLld]
  float* X = lds + NB * kLld;    // [NB][kXld]
  const int t = threadIdx.x, c = t & 63, rg = t >> 6;
  for (int e = t; e < NB * NB; e += 256) L[(e / NB) * kLld + e % NB] = A[(int64_t)(k0 + e / NB) * lda + k0 + e % NB];
  const int col = c0 + blockIdx.x * kTile + c;
  const bool ok = col < c0 + ncols;
  for (int i = rg; i < NB; i += 4) X[i * kXld + c] = ok ? A[(int64_t)(k0 + i) * lda + col] : 0.0f;
  __syncthreads();
  tile_lower_solve<true>(X, L, nullptr);
  if (ok)
    for (int i = rg; i < NB; i += 4) A[(int64_t)(k0 + i) * lda + col] = X[i * kXld + c];
}

// L21 = A21 U11^-1 in place for rows [r0, r0 + nrows), 64 per workgroup.
__global__ __launch_bounds__(256) void trsm_l21_kernel(float* __restrict__ A, int64_t lda, int k0, int r0, int nrows) {
  extern __shared__ float lds[];
  float* L = lds;                    // [NB][kLld]: L[i][k] = U11[k][i]
  float* X = lds + NB * kLld;        // [NB][kXld]: X[i][c] = A21[row c][i]
  float* rinv = X + NB * kXld;       // [NB]
  const int t = threadIdx.x;
  for (int e = t; e < NB * NB; e += 256) {
    const int k = e / NB, i = e % NB;  // coalesced along U11's row k
    L[i * kLld + k] = A[(int64_t)(k0 + k) * lda + k0 + i];
  }
  if (t < NB) rinv[t] = 1.0f / A[(int64_t)(k0 + t) * lda + k0 + t];
  const int rbase = r0 + blockIdx.x * kTile;
  for (int e = t; e < kTile * NB; e += 256) {
    const int c = e / NB, i = e % NB;  // coalesced along the row of A21
    const int row = rbase + c;
    X[i * kXld + c] = row < r0 + nrows ? A[(int64_t)row * lda + k0 + i] : 0.0f;
  }
  __syncthreads();
  tile_lower_solve<false>(X, L, rinv);
  for (int e = t; e < kTile * NB; e += 256) {
    const int c = e / NB, i = e % NB;
    const int row = rbase + c;
    if (row < r0 + nrows) A[(int64_t)row * lda + k0 + i] = X[i * kXld + c];
  }
}

}  // namespace
}  // namespace gelim

struct gelim_mixed_plan {
  int64_t n = 0, np = 0, ldm = 0;
  float* M = nullptr;       // np x ldm: the transformed matrix, then its LU factors
  double* ud = nullptr;     // U's butterfly diagonals (8 x np/4)
  double* vd = nullptr;     // V's
  unsigned* flags = nullptr;  // forward substitution hand-off flags (np / 64 + 2)
  double* c = nullptr;      // U^T r (np)
  float* y = nullptr;       // L^-1 c (np, fp32)
  double* z = nullptr;      // U^-1 y (np)
  double* yw = nullptr;     // back-substitution workspace (np + 2)
  int* info = nullptr;
};

extern "C" int64_t gelim_mixed_max_n(void) { return 16384; }

extern "C" void gelim_mixed_plan_destroy(gelim_mixed_plan* p) {
  if (!p) return;
  for (void* q : {(void*)p->M, (void*)p->ud, (void*)p->vd, (void*)p->flags, (void*)p->c, (void*)p->y, (void*)p->z,
                  (void*)p->yw, (void*)p->info})
    (void)hipFree(q);
  delete p;
}

// n: order of the system; ud / vd: host arrays of 8 * np/4 butterfly entries
// each (np = gelim_mixed_padded(n)), exp(r/10) with r uniform in [-1/2, 1/2].
extern "C" int64_t gelim_mixed_padded(int64_t n) { return (n + gelim::kPadTo - 1) / gelim::kPadTo * gelim::kPadTo; }

extern "C" gelim_mixed_plan* gelim_mixed_plan_create(int64_t n, const double* ud, const double* vd) {
  const int64_t np = gelim_mixed_padded(n);
  if (n <= 0 || np > gelim_mixed_max_n()) {
    GELIM_FAIL(GELIM_E_ARG, "mixed plan: n must be in [1, " + std::to_string(gelim_mixed_max_n()) +
                                "] (persistent triangular solves: every 64-row block resident)");
    return nullptr;
  }
  auto* p = new gelim_mixed_plan;
  p->n = n;
  p->np = np;
  p->ldm = np + 4;  // 16-byte rows, off the power-of-two stride
  auto fail = [&](const char* what) -> gelim_mixed_plan* {
    GELIM_FAIL(GELIM_E_NOMEM, std::string("mixed plan: ") + what);
    gelim_mixed_plan_destroy(p);
    return nullptr;
  };
  const size_t nd = (size_t)2 * np;  // 8 arrays of np/4
  if (hipMalloc((void**)&p->M, sizeof(float) * (size_t)np * p->ldm) != hipSuccess) return fail("matrix");
  if (hipMalloc((void**)&p->ud, sizeof(double) * nd) != hipSuccess) return fail("ud");
  if (hipMalloc((void**)&p->vd, sizeof(double) * nd) != hipSuccess) return fail("vd");
  if (hipMalloc((void**)&p->flags, sizeof(unsigned) * (np / 64 + 2)) != hipSuccess) return fail("flags");
  if (hipMalloc((void**)&p->c, sizeof(double) * np) != hipSuccess) return fail("c");
  if (hipMalloc((void**)&p->y, sizeof(float) * np) != hipSuccess) return fail("y");
  if (hipMalloc((void**)&p->z, sizeof(double) * np) != hipSuccess) return fail("z");
  if (hipMalloc((void**)&p->yw, sizeof(double) * (np + 2)) != hipSuccess) return fail("yw");
  if (hipMalloc((void**)&p->info, 16) != hipSuccess) return fail("info");
  if (hipMemcpy(p->ud, ud, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("ud copy");
  if (hipMemcpy(p->vd, vd, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("vd copy");
  return p;
}

// Transform the augmented fp64 system's matrix (n x n at aug, leading
// dimension ld) into the plan's fp32 matrix and factor it without pivoting.
// Returns 0, or 1 + the first column whose pivot is zero / not finite (the
// caller then falls back to partial pivoting); < 0 on errors.  Synchronises.
extern "C" int gelim_mixed_factor(gelim_mixed_plan* p, const double* aug, int64_t ld, void* stream) {
  using namespace gelim;
  if (!p || !aug) return GELIM_FAIL(GELIM_E_ARG, "mixed_factor: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t np = p->np, h = np / 4, ldm = p->ldm;
  HIP_TRY(hipMemsetAsync(p->info, 0x7f, 4, s));  // INT_MAX-ish: atomicMin keeps the first bad column
  hipLaunchKernelGGL(rbt_matrix_kernel, dim3((unsigned)((h + 255) / 256), (unsigned)h), dim3(256), 0, s, aug, ld,
                     (int)p->n, (int)np, p->ud, p->vd, p->M, ldm);
  HIP_TRY(hipGetLastError());
  static const bool attr = [] {
    const int diag = (int)(sizeof(float) * NB * kLdsLd), tr = (int)(sizeof(float) * (NB * kLld + NB * kXld + NB));
    return hipFuncSetAttribute((const void*)diag_lu_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, diag) ==
               hipSuccess &&
           hipFuncSetAttribute((const void*)trsm_u12_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, tr) ==
               hipSuccess &&
           hipFuncSetAttribute((const void*)trsm_l21_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, tr) ==
               hipSuccess;
  }();
  if (!attr) return GELIM_FAIL(GELIM_E_HIP, "mixed_factor: LDS attributes refused");
  float* M = p->M;
  for (int64_t k0 = 0; k0 < np; k0 += NB) {
    hipLaunchKernelGGL(diag_lu_kernel, dim3(1), dim3(1024), sizeof(float) * NB * kLdsLd, s, M, ldm, (int)k0, p->info);
    HIP_TRY(hipGetLastError());
    const int64_t rest = np - k0 - NB;
    if (rest <= 0) break;
    const unsigned g = (unsigned)((rest + kTile - 1) / kTile);
    const size_t tr = sizeof(float) * (NB * kLld + NB * kXld + NB);
    hipLaunchKernelGGL(trsm_u12_kernel, dim3(g), dim3(256), tr, s, M, ldm, (int)k0, (int)(k0 + NB), (int)rest);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(trsm_l21_kernel, dim3(g), dim3(256), tr, s, M, ldm, (int)k0, (int)(k0 + NB), (int)rest);
    HIP_TRY(hipGetLastError());
    // A22 -= L21 U12 (fp32 MFMA, K = NB)
    float* A22 = M + (k0 + NB) * ldm + k0 + NB;
    GELIM_TRY(matmul_f32(M + (k0 + NB) * ldm + k0, ldm, M + k0 * ldm + k0 + NB, ldm, A22, ldm, rest, rest, NB, 1,
                         GELIM_MM_MFMA, s, -1.0f));
  }
  int h_info = 0;
  HIP_TRY(hipMemcpyAsync(&h_info, p->info, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return h_info == 0x7f7f7f7f ? 0 : h_info;
}

// d = V (LU)^-1 U^T [r; 0]: the correction of one refinement step (r, d:
// n fp64 entries, r with stride incr).
extern "C" int gelim_mixed_apply(gelim_mixed_plan* p, const double* r, int64_t incr, double* d, void* stream) {
  using namespace gelim;
  if (!p || !r || !d) return GELIM_FAIL(GELIM_E_ARG, "mixed_apply: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t np = p->np, h = np / 4;
  const unsigned g = (unsigned)((h + 255) / 256);
  hipLaunchKernelGGL(rbt_vec_kernel, dim3(g), dim3(256), 0, s, r, incr, (int)p->n, (int)np, p->ud, 1, p->c);
  HIP_TRY(hipGetLastError());
  GELIM_TRY(fwdsub_unit_f32(p->M, p->ldm, p->c, p->y, np, p->z, p->flags, s));
  GELIM_TRY(backsub_f32(p->M, p->ldm, p->y, 1, p->z, nullptr, np, 0, p->yw, s, nullptr, nullptr));
  // x = V z, only the first n entries are kept (the padding's are zero in exact arithmetic)
  hipLaunchKernelGGL(rbt_vec_kernel, dim3(g), dim3(256), 0, s, p->z, (int64_t)1, (int)np, (int)np, p->vd, 0, p->c);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(d, p->c, sizeof(double) * p->n, hipMemcpyDeviceToDevice, s));
  return GELIM_OK;
}

extern "C" int64_t gelim_mixed_plan_np(const gelim_mixed_plan* p) { return p ? p->np : 0; }
