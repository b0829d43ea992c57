// Randomised no-pivoting engines (GaussSolver backends "hip-mixed" and
// "hip-rbt"): a random butterfly transform (RBT) of the system, a NO-pivoting
// blocked LU of the transformed matrix on the matrix cores -- fp32 factors
// ("hip-mixed") or fp64 factors ("hip-rbt") -- and fp64 iterative refinement
// against the original system (the loop is in models/gauss_solver.py; when it
// does not reach the fp64 error class the solver falls back to the fp64
// partial-pivoting engine by itself).
//
// Why: every exact partial-pivoting engine here is bound by its pivot chain
// (one global arg-max per column: ~3 us per column on the wide-panel leaves
// at n = 8192, profiles/leaf_fused_vs_2hop.txt).  A two-sided recursive
// butterfly transform U^T A V (Parker 1995; Baboulin, Dongarra et al. 2013)
// makes pivoting unnecessary with probability close to one, and without
// pivoting the factorisation has no per-column global reduction at all.  The
// reference's loop (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182,
// fp64, partial pivoting) is what the refinement answers to: the residual is
// always taken in fp64 on the ORIGINAL system.
//
// Factorisation (T = float or double): block LDU without pivoting, 128-column
// blocks.  Per block k:
//  * diag_inv_kernel: ONE workgroup inverts the (Schur) diagonal block A_kk
//    by Gauss-Jordan in fp64 registers (8 x 8 tiles per thread, one uniform
//    rank-1 update and one barrier per column) -> Dinv_k (kept for the solves);
//  * W = A_kk^-1 A_k,rest and A_rest,rest -= A_rest,k W on the matrix cores
//    (fp64 dgemm.hip v_mfma_f64_16x16x4f64, or fp32 gemm_f32.hip
//    v_mfma_f32_32x32x2f32 with a rounded copy of the inverse).  A_rest,k and
//    A_k,rest stay in place as the factor's off-diagonal blocks.
// The fp32 engine still inverts in fp64: an fp32 Gauss-Jordan of a no-pivoting
// block with cond ~1e7 would be useless, while a correctly rounded copy of an
// accurate inverse only costs eps32 relative in W.
//
// Solves (blk_trsv_kernel, one persistent launch per direction): workgroup w
// owns block row b (128 equations); it applies the solved blocks before it in
// chain order (the next block's factor loads in flight under the current
// block's FMAs), then multiplies by the stored inverse -- a mat-vec, not a
// 128-step chain -- in fp64 arithmetic over the T factor, and publishes its
// block as plain agent-scope stores into a buffer pre-filled with a
// signalling-NaN sentinel: the consumer polls the values themselves, so a
// hand-off is one store + one load (no drain, barrier or flag).  Spins are
// bounded (200 ms) and report through an error word.
//
// Depth-2 recursive butterfly: W = L1 L0, L0 = B<n> = 1/sqrt2 [R S; R -S]
// on (i, i + n/2), L1 = diag(B<n/2>_a, B<n/2>_b) on (i, i + n/4) and
// (i + n/2, i + 3n/4); R, S diagonal with entries exp(r / 10), r uniform in
// [-1/2, 1/2].  Both levels act on the index groups {i, i + h, i + 2h,
// i + 3h} (h = n/4) as one 4 x 4 matrix W_i, so M = U^T A V is ONE pass over
// A: every 4 x 4 group of entries becomes U_i^T A_g V_j.  The system is
// padded to np = a multiple of 128 with an identity block (b padded with
// zeros).  Storage: the block-LDU factor overwrites the transformed matrix
// (diagonal blocks unused, their inverses in Dinv).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <utility>

#include "device_common.h"
#include "gelim/internal.h"
#include "rbt.h"

namespace gelim {
int matmul_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int64_t N,
               int64_t K, int accumulate, int kernel, hipStream_t s, float alpha, double* C64);
int dgemm_ex(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
             int64_t N, int64_t K, double alpha, int accumulate, hipStream_t s);
int dgemm_capped(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate);
int residual_f64(const double* aug, int64_t ld, int64_t n, const double* x, double* r, hipStream_t s, int matvec,
                 double* w);

namespace {

constexpr int NB = 128;         // LU block = solve block
constexpr int kPadTo = NB;      // np multiple
constexpr int kDT = 512;        // solve workgroup: 128 rows x 4 column quarters
constexpr int kQW = NB / 4;     // columns per quarter
constexpr int kMaxBlocks = 256;  // persistent solves: every block row resident
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

using rbt::group_w;

// M[g] = U_i^T A_g V_j for every 4 x 4 group; A is the n x n system (row
// major, lda), padded on the fly to np with an identity block.
template <typename T>
__global__ __launch_bounds__(256) void rbt_matrix_kernel(const double* __restrict__ A, int64_t lda, int n, int np,
                                                        const double* __restrict__ ud, const double* __restrict__ vd,
                                                        T* __restrict__ M, int64_t ldm) {
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
      M[(int64_t)(i + q * h) * ldm + j + p * h] = (T)v;
    }
}

// out = U^T [b; 0] (left) or out = V y (right), fp64 vectors of np entries
// (b: n entries with stride incb; the padding reads as 0)
__global__ __launch_bounds__(256) void rbt_vec_kernel(const double* __restrict__ b, int64_t incb, int n, int np,
                                                     const double* __restrict__ d, int transpose,
                                                     double* __restrict__ out, int nout) {
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
    if (i + q * h < nout) out[i + q * h] = s;
  }
}

// ---- diagonal block inverse: Gauss-Jordan without pivoting ---------------------
// Block LDU (no pivoting): A = [I 0; A21 A11^-1 I] [A11 A12; 0 S], S = A22 -
// A21 (A11^-1 A12).  So a block step needs only A11^-1 (kept, fp64, for the
// solves) and two GEMMs, W = A11^-1 A12 and A22 -= A21 W; A21 / A12 stay in
// place as the factor's off-diagonal blocks.
//
// One workgroup of 256 threads (one wave per SIMD) inverts the 128 x 128
// block in place in registers: thread (rg, cg) = (t >> 4, t & 15) holds the
// 8 x 8 tile rows 8 rg.., columns 8 cg...  Step k of Gauss-Jordan is ONE
// uniform rank-1 update of the whole block,
//   a[i][j] -= g_i u_j,  g_i = a[i][k] - [i == k],  u_j = a[k][j] / a[k][k] (j != k),  u_k = 1 + 1 / a[k][k],
// which gives a'[k][k] = 1/a_kk, a'[k][j] = a_kj/a_kk, a'[i][k] = -a_ik/a_kk
// and the Schur update elsewhere with no special cases.  Row k and column k
// are published raw through parity-buffered LDS one step ahead (one barrier
// per step), and the step loop is unrolled by 8 so every in-tile index (k % 8)
// is static: publishing is a predicated store, not a register pick.  ~500
// cycles per step, 128 steps: 72 us per block (the earlier LU + two
// triangular-inverse loops with one row per lane: 330 us, instruction-bound;
// a 4-column blocked Gauss-Jordan step -- explicit 4 x 4 pivot-block inverse,
// rank-4 update -- was slower, 81 us, and lost accuracy: refinement needed
// more corrections and fell back at n >= 4096).
constexpr int kTl = 8;    // tile columns (and rows, TR = 8)

// Row k / column k as 16 chunks of 8 doubles at a stride of 10: a
// ds_read_b128 lane group reads all 16 chunks at once (16 distinct column
// groups), and at a stride of 8 they fell on 4 bank sets (4-way, 42 % of the
// kernel's LDS cycles, profiles/pmc_rbt_8192.txt); at 10 (80 B = 20 banks)
// they tile the 64 banks exactly.
constexpr int kGjStride = kTl + 2;
constexpr int gj_at(int i) { return (i / kTl) * kGjStride + i % kTl; }

template <typename TI>
struct alignas(16) GjLds {
  TI row[2][NB / kTl * kGjStride];
  TI col[2][NB / kTl * kGjStride];
};

// 1 / pivot: v_rcp_f64 + two Newton steps (within an ulp of the IEEE
// quotient; the refinement absorbs the rest) -- 3 dependent FMAs instead of
// the ~8-deep IEEE division sequence on the critical path of every column
__device__ __forceinline__ double gj_recip(double piv) {
  double pk = __builtin_amdgcn_rcp(piv);
  pk = fma(pk, fma(-piv, pk, 1.0), pk);
  return fma(pk, fma(-piv, pk, 1.0), pk);
}

// Step k = 8 kg + KK of the Gauss-Jordan inverse on TR x 8 tiles (TR = 8:
// 256 threads, one wave per SIMD; TR = 4: 512 threads, two waves per SIMD).
// The raw row / column are published and every thread scales after the
// barrier (publishing u and g ready to use -- the reciprocal taken from the
// pivot's lane by v_readlane in the publishing wave -- made the factor 7 %
// slower: the publisher's longer path before its bulk update is the
// critical one, profiles/rbt_engine_round3.txt).
template <int TR, int KK>
__device__ __forceinline__ void gj_step(double (&a)[TR][kTl], GjLds<double>& sh, int kg, int rg, int cg) {
  const int k = kTl * kg + KK;
  constexpr int par = KK & 1;  // kTl is even: k and KK share parity
  constexpr int RPG = kTl / TR;  // row groups per column group
  const double pk = gj_recip(sh.row[par][gj_at(k)]);
  double u[kTl], g[TR];
#pragma unroll
  for (int j = 0; j < kTl; j += 2) {
    const double2 v = *reinterpret_cast<const double2*>(&sh.row[par][kGjStride * cg + j]);
    u[j] = v.x * pk;
    u[j + 1] = v.y * pk;
  }
#pragma unroll
  for (int i = 0; i < TR; i += 2) {
    const double2 v = *reinterpret_cast<const double2*>(&sh.col[par][gj_at(TR * rg) + i]);
    g[i] = v.x;
    g[i + 1] = v.y;
  }
  u[KK] = (cg == kg) ? 1.0 + pk : u[KK];
  g[KK % TR] -= (rg == RPG * kg + KK / TR) ? 1.0 : 0.0;
  // next step's pivot row (in-tile row r1 of row group rg1) and column
  constexpr int kk1 = (KK + 1) % kTl;
  constexpr int r1 = (KK + 1) % TR;
  const int kg1 = KK + 1 == kTl ? kg + 1 : kg;
  const int rg1 = (k + 1) / TR;
  const bool more = k + 1 < NB;
  // the next step's pivot row / column first: their LDS stores then drain
  // under the bulk of the update instead of after it
#pragma unroll
  for (int j = 0; j < kTl; ++j) a[r1][j] = fma(-g[r1], u[j], a[r1][j]);
#pragma unroll
  for (int i = 0; i < TR; ++i)
    if (i != r1) a[i][kk1] = fma(-g[i], u[kk1], a[i][kk1]);
  if (more && rg == rg1) {
#pragma unroll
    for (int j = 0; j < kTl; j += 2)
      *reinterpret_cast<double2*>(&sh.row[par ^ 1][kGjStride * cg + j]) = make_double2(a[r1][j], a[r1][j + 1]);
  }
  if (more && cg == kg1) {
#pragma unroll
    for (int i = 0; i < TR; i += 2)
      *reinterpret_cast<double2*>(&sh.col[par ^ 1][gj_at(TR * rg) + i]) = make_double2(a[i][kk1], a[i + 1][kk1]);
  }
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int j = 0; j < kTl; ++j)
      if (i != r1 && j != kk1) a[i][j] = fma(-g[i], u[j], a[i][j]);
  __syncthreads();
}

template <int TR, int... KK>
__device__ __forceinline__ void gj_steps(double (&a)[TR][kTl], GjLds<double>& sh, int kg, int rg, int cg,
                                         std::integer_sequence<int, KK...>) {
  (gj_step<TR, KK>(a, sh, kg, rg, cg), ...);
}

// Dinv = Ablk^-1 (fp64, row-major NB x NB) of the NB x NB T block at Ablk
// (leading dimension lda); with Tinv, also a T copy (the fp32 engine's GEMM
// operand).  The block is read, not modified.  info: atomicMin of 1 + k0 (the
// block's first global column) when the inverse is not finite (a zero / tiny
// pivot).
template <typename T, int TR>
__global__ __launch_bounds__(16 * NB / TR) void diag_inv_kernel(const T* __restrict__ Ablk, int64_t lda, int k0,
                                                               double* __restrict__ Dinv, T* __restrict__ Tinv,
                                                               int* __restrict__ info) {
  __shared__ GjLds<double> sh;
  const int t = threadIdx.x, rg = t >> 4, cg = t & 15;
  double a[TR][kTl];
#pragma unroll
  for (int i = 0; i < TR; ++i) {
    const T* src = Ablk + (int64_t)(TR * rg + i) * lda + kTl * cg;
#pragma unroll
    for (int j = 0; j < kTl; ++j) a[i][j] = (double)src[j];
  }
  if (rg == 0) {
#pragma unroll
    for (int j = 0; j < kTl; ++j) sh.row[0][kGjStride * cg + j] = a[0][j];
  }
  if (cg == 0) {
#pragma unroll
    for (int i = 0; i < TR; ++i) sh.col[0][gj_at(TR * rg) + i] = a[i][0];
  }
  __syncthreads();
  for (int kg = 0; kg < NB / kTl; ++kg) gj_steps<TR>(a, sh, kg, rg, cg, std::make_integer_sequence<int, kTl>{});
  bool fin = true;
#pragma unroll
  for (int i = 0; i < TR; ++i) {
    double* dst = Dinv + (int64_t)(TR * rg + i) * NB + kTl * cg;
#pragma unroll
    for (int j = 0; j < kTl; ++j) {
      fin = fin && isfinite(a[i][j]);
      dst[j] = a[i][j];
    }
    if (Tinv) {
      T* tdst = Tinv + (int64_t)(TR * rg + i) * NB + kTl * cg;
#pragma unroll
      for (int j = 0; j < kTl; ++j) tdst[j] = (T)a[i][j];
    }
  }
  if (!fin) atomicMin(info, k0 + 1);
}

// ---- two Gauss-Jordan steps per barrier ----------------------------------------
// The same uniform rank-1 steps, paired: rows k, k+1 and columns k, k+1 of
// the block are published raw (before step k) behind ONE barrier, and every
// thread derives step k+1's operands itself -- column k+1 and row k+1 after
// step k are one FMA each from the published values (c1_i = a_i,k+1 - g_i
// u_k+1, r1_j = a_k+1,j - g_k+1 u_j, pivot a_k+1,k+1 - g_k+1 u_k+1), exactly
// the FMAs their owners perform in the one-step form -- then applies
// a -= g u^T + g' u'^T.  Every element sees the same operation sequence as
// in diag_inv_kernel (bit-identical results) with half the barriers.
template <typename TI>
struct alignas(16) GjPairLds {
  TI row[2][2][NB / kTl * kGjStride];  // [parity][row k / k+1]
  TI col[2][2][NB / kTl * kGjStride];  // [parity][column k / k+1]
};

template <int TR, int KK>  // KK even: pair (k, k+1), k = 8 kg + KK
__device__ __forceinline__ void gj_pair(double (&a)[TR][kTl], GjPairLds<double>& sh, int kg, int rg, int cg) {
  static_assert(KK % 2 == 0 && TR % 2 == 0, "pairs of rows share a tile");
  const int k = kTl * kg + KK;
  constexpr int par = (KK / 2) & 1;  // kTl / 2 pairs per tile: even, so the parity is static
  constexpr int RPG = kTl / TR;
  const double akk = sh.row[par][0][gj_at(k)];
  const double ak1 = sh.row[par][0][gj_at(k + 1)];  // a[k][k+1]
  const double a1k = sh.row[par][1][gj_at(k)];      // a[k+1][k]
  const double a11 = sh.row[par][1][gj_at(k + 1)];
  const double pk = gj_recip(akk);
  double u[kTl], g[TR], u1[kTl], g1[TR];
#pragma unroll
  for (int j = 0; j < kTl; j += 2) {
    const double2 v = *reinterpret_cast<const double2*>(&sh.row[par][0][kGjStride * cg + j]);
    const double2 w = *reinterpret_cast<const double2*>(&sh.row[par][1][kGjStride * cg + j]);
    u[j] = v.x * pk;
    u[j + 1] = v.y * pk;
    u1[j] = w.x;
    u1[j + 1] = w.y;
  }
#pragma unroll
  for (int i = 0; i < TR; i += 2) {
    const double2 v = *reinterpret_cast<const double2*>(&sh.col[par][0][gj_at(TR * rg) + i]);
    const double2 w = *reinterpret_cast<const double2*>(&sh.col[par][1][gj_at(TR * rg) + i]);
    g[i] = v.x;
    g[i + 1] = v.y;
    g1[i] = w.x;
    g1[i + 1] = w.y;
  }
  const bool kcol = cg == kg;                   // columns k, k+1 are in this thread's tile
  const bool krow = rg == RPG * kg + KK / TR;  // rows k, k+1 are
  u[KK] = kcol ? 1.0 + pk : u[KK];
  g[KK % TR] -= krow ? 1.0 : 0.0;
  // step k applied to column k+1 (rows of this tile), row k+1 (columns of
  // this tile) and the next pivot
  const double uk1 = ak1 * pk;  // u[k+1]
  const double gk1 = a1k;       // g[k+1]
#pragma unroll
  for (int i = 0; i < TR; ++i) g1[i] = fma(-g[i], uk1, g1[i]);
#pragma unroll
  for (int j = 0; j < kTl; ++j) u1[j] = fma(-gk1, u[j], u1[j]);
  const double pk1 = gj_recip(fma(-gk1, uk1, a11));
#pragma unroll
  for (int j = 0; j < kTl; ++j) u1[j] *= pk1;
  u1[KK + 1] = kcol ? 1.0 + pk1 : u1[KK + 1];
  g1[(KK + 1) % TR] -= krow ? 1.0 : 0.0;
  // the next pair's rows / columns first, published raw
  constexpr int KN = (KK + 2) % kTl;
  constexpr int rn = KN % TR;
  const int kgn = KK + 2 == kTl ? kg + 1 : kg;
  const int rgn = (k + 2) / TR;
  const bool more = k + 2 < NB;
#pragma unroll
  for (int j = 0; j < kTl; ++j) {
    a[rn][j] = fma(-g1[rn], u1[j], fma(-g[rn], u[j], a[rn][j]));
    a[rn + 1][j] = fma(-g1[rn + 1], u1[j], fma(-g[rn + 1], u[j], a[rn + 1][j]));
  }
#pragma unroll
  for (int i = 0; i < TR; ++i)
    if (i != rn && i != rn + 1) {
      a[i][KN] = fma(-g1[i], u1[KN], fma(-g[i], u[KN], a[i][KN]));
      a[i][KN + 1] = fma(-g1[i], u1[KN + 1], fma(-g[i], u[KN + 1], a[i][KN + 1]));
    }
  if (more && rg == rgn) {
#pragma unroll
    for (int j = 0; j < kTl; j += 2) {
      *reinterpret_cast<double2*>(&sh.row[par ^ 1][0][kGjStride * cg + j]) = make_double2(a[rn][j], a[rn][j + 1]);
      *reinterpret_cast<double2*>(&sh.row[par ^ 1][1][kGjStride * cg + j]) =
          make_double2(a[rn + 1][j], a[rn + 1][j + 1]);
    }
  }
  if (more && cg == kgn) {
#pragma unroll
    for (int i = 0; i < TR; i += 2) {
      *reinterpret_cast<double2*>(&sh.col[par ^ 1][0][gj_at(TR * rg) + i]) = make_double2(a[i][KN], a[i + 1][KN]);
      *reinterpret_cast<double2*>(&sh.col[par ^ 1][1][gj_at(TR * rg) + i]) =
          make_double2(a[i][KN + 1], a[i + 1][KN + 1]);
    }
  }
#pragma unroll
  for (int i = 0; i < TR; ++i)
#pragma unroll
    for (int j = 0; j < kTl; ++j)
      if (i != rn && i != rn + 1 && j != KN && j != KN + 1)
        a[i][j] = fma(-g1[i], u1[j], fma(-g[i], u[j], a[i][j]));
  __syncthreads();
}

template <int TR, int... KK>
__device__ __forceinline__ void gj_pairs(double (&a)[TR][kTl], GjPairLds<double>& sh, int kg, int rg, int cg,
                                         std::integer_sequence<int, KK...>) {
  (gj_pair<TR, 2 * KK>(a, sh, kg, rg, cg), ...);
}

template <int TR>
__global__ __launch_bounds__(16 * NB / TR) void diag_inv_pair_kernel(const double* __restrict__ Ablk, int64_t lda,
                                                                    int k0, double* __restrict__ Dinv,
                                                                    int* __restrict__ info) {
  __shared__ GjPairLds<double> sh;
  const int t = threadIdx.x, rg = t >> 4, cg = t & 15;
  double a[TR][kTl];
#pragma unroll
  for (int i = 0; i < TR; ++i) {
    const double* src = Ablk + (int64_t)(TR * rg + i) * lda + kTl * cg;
#pragma unroll
    for (int j = 0; j < kTl; ++j) a[i][j] = src[j];
  }
  if (rg == 0) {
#pragma unroll
    for (int j = 0; j < kTl; ++j) {
      sh.row[0][0][kGjStride * cg + j] = a[0][j];
      sh.row[0][1][kGjStride * cg + j] = a[1][j];
    }
  }
  if (cg == 0) {
#pragma unroll
    for (int i = 0; i < TR; ++i) {
      sh.col[0][0][gj_at(TR * rg) + i] = a[i][0];
      sh.col[0][1][gj_at(TR * rg) + i] = a[i][1];
    }
  }
  __syncthreads();
  for (int kg = 0; kg < NB / kTl; ++kg)
    gj_pairs<TR>(a, sh, kg, rg, cg, std::make_integer_sequence<int, kTl / 2>{});
  bool fin = true;
#pragma unroll
  for (int i = 0; i < TR; ++i) {
    double* dst = Dinv + (int64_t)(TR * rg + i) * NB + kTl * cg;
#pragma unroll
    for (int j = 0; j < kTl; ++j) {
      fin = fin && isfinite(a[i][j]);
      dst[j] = a[i][j];
    }
  }
  if (!fin) atomicMin(info, k0 + 1);
}

// ---- blocked Gauss-Jordan inverse on the matrix cores ------------------------
// The same inverse, blocked: block steps of KB = 32 (or 16) pivots.  The 128 x 128
// block lives in LDS (133 KB of the CU's 160 KB); per block step b (rows /
// columns kb = 32 b ..):
//  1. wave 0 inverts the 32 x 32 pivot block in place by the unblocked
//     Gauss-Jordan step above (the uniform rank-1 form; lane l holds row
//     l / 2, half l % 2 of the columns; the pivot row goes through a
//     wave-private LDS line, the pivot column through one DPP lane swap);
//  2. the pivot rows: A[kb, j] = P^-1 A[kb, j] for j outside kb;
//  3. every other row: A[i, j] -= A[i, kb] A[kb, j] (j outside kb) and
//     A[i, kb] = -A[i, kb] P^-1 -- one GEMM with the pivot block columns of
//     the right operand = P^-1 and of the start value = 0.
// Steps 2 and 3 run on v_mfma_f64_16x16x4f64 (16 x 16 tiles, K = 32, every
// wave one column tile of 6 row tiles in step 3), results held in registers
// across a barrier, then stored (the GEMMs read what they overwrite).  The
// 2.1 M FMAs of the inverse move from 128 barrier-separated VALU rank-1
// steps to 8 MFMA phases + 128 single-wave steps on 32 x 32.
constexpr int kBjLd = NB + 2;  // LDS row stride (doubles): 16 rows of an operand load hit distinct banks
constexpr int kBjThreads = 512;

struct BjLds {
  double a[NB * kBjLd];
  double rowb[2][32];
};

template <int CTRL>
__device__ __forceinline__ double mov_dpp_f64(double x) {
  const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)__double_as_longlong(x), CTRL, 0xf, 0xf,
                                                         false);
  const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp(
      (int)(unsigned)((uint64_t)__double_as_longlong(x) >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// step 1: wave 0 inverts the KB x KB pivot block at (kb, kb) in place.  Lane
// l holds row l / LPR, columns VPL (l % LPR) .. of it (LPR = 64 / KB lanes per
// row, VPL = KB / LPR values each): the pivot row goes through a
// wave-private LDS line, the pivot column's entry of a row through one DPP
// move inside the row's lane group.  Step K (compile time) of it:
template <int KB, int K>
__device__ __forceinline__ void bj_leaf_step(BjLds& sh, double (&p)[KB * KB / 64], int r, int cg) {
  constexpr int LPR = 64 / KB, VPL = KB / LPR;
  double* rb = sh.rowb[K & 1];
  if (r == K) {
#pragma unroll
    for (int j = 0; j < VPL; j += 2) *reinterpret_cast<double2*>(rb + VPL * cg + j) = make_double2(p[j], p[j + 1]);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-private line: in-order LDS
  double v[VPL];
#pragma unroll
  for (int j = 0; j < VPL; j += 2) {
    const double2 w = *reinterpret_cast<const double2*>(rb + VPL * cg + j);
    v[j] = w.x;
    v[j + 1] = w.y;
  }
  const double akk = rb[K];
  // my row's entry in column K: lane-group member K / VPL, register K % VPL
  double gk;
  if constexpr (LPR == 2) {
    const double own = p[K % VPL];
    const double oth = mov_dpp_f64<0xB1>(own);  // quad_perm [1,0,3,2]: the other lane of the pair
    gk = (cg == K / VPL) ? own : oth;
  } else {  // LPR == 4: the quad is the row's lane group
    constexpr int src = K / VPL;
    gk = mov_dpp_f64<src | (src << 2) | (src << 4) | (src << 6)>(p[K % VPL]);
  }
  const double g = gk - (r == K ? 1.0 : 0.0);
  const double pk = gj_recip(akk);
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const double u = (VPL * cg + j == K) ? 1.0 + pk : v[j] * pk;
    p[j] = fma(-g, u, p[j]);
  }
}

template <int KB, int... K>
__device__ __forceinline__ void bj_leaf_steps(BjLds& sh, double (&p)[KB * KB / 64], int r, int cg,
                                              std::integer_sequence<int, K...>) {
  (bj_leaf_step<KB, K>(sh, p, r, cg), ...);
}

template <int KB>
__device__ __forceinline__ void bj_leaf(BjLds& sh, int kb, int lane) {
  constexpr int LPR = 64 / KB, VPL = KB / LPR;
  const int r = lane / LPR, cg = lane % LPR;
  double* prow = &sh.a[(kb + r) * kBjLd + kb + VPL * cg];
  double p[VPL];
#pragma unroll
  for (int j = 0; j < VPL; j += 2) {
    const double2 v = *reinterpret_cast<const double2*>(prow + j);
    p[j] = v.x;
    p[j + 1] = v.y;
  }
  bj_leaf_steps<KB>(sh, p, r, cg, std::make_integer_sequence<int, KB>{});
#pragma unroll
  for (int j = 0; j < VPL; j += 2) *reinterpret_cast<double2*>(prow + j) = make_double2(p[j], p[j + 1]);
}

// the c-th 16-row / column tile outside the pivot block [kb, kb + KB)
template <int KB>
__device__ __forceinline__ int bj_outside(int c, int kb) { return 16 * c < kb ? 16 * c : 16 * c + KB; }

template <int KB>
__global__ __launch_bounds__(kBjThreads) void bj_inv_kernel(const double* __restrict__ Ablk, int64_t lda, int k0,
                                                            double* __restrict__ Dinv, int* __restrict__ info) {
  constexpr int RT = KB / 16;          // row tiles of the pivot rows
  constexpr int OT = (NB - KB) / 16;   // tiles outside the pivot block
  __shared__ BjLds sh;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m = lane & 15, q = lane >> 4;
  {  // lanes along a row: coalesced
    const int c = t & (NB - 1);
#pragma unroll 8
    for (int r = t >> 7; r < NB; r += kBjThreads / NB) sh.a[r * kBjLd + c] = Ablk[(int64_t)r * lda + c];
  }
  __syncthreads();
  for (int kb = 0; kb < NB; kb += KB) {
    if (wave == 0) bj_leaf<KB>(sh, kb, lane);
    __syncthreads();
    // step 2: RT x OT tiles of the pivot rows, dealt to the waves
    constexpr int N2 = (RT * OT + 7) / 8;
    dev::d4 acc2[N2];
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int ti = wave + 8 * u;
      if (ti < RT * OT) {
        const int r0 = kb + 16 * (ti / OT), c0 = bj_outside<KB>(ti % OT, kb);
        dev::d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < KB; kk += 4) {
          const double av = sh.a[(r0 + m) * kBjLd + kb + kk + q];   // P^-1 (row r0 + m, col kb + k)
          const double bv = sh.a[(kb + kk + q) * kBjLd + c0 + m];   // A[kb + k, c0 + n]
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
        acc2[u] = acc;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < N2; ++u) {
      const int ti = wave + 8 * u;
      if (ti < RT * OT) {
        const int r0 = kb + 16 * (ti / OT), c0 = bj_outside<KB>(ti % OT, kb);
#pragma unroll
        for (int i = 0; i < 4; ++i) sh.a[(r0 + q + 4 * i) * kBjLd + c0 + m] = acc2[u][i];
      }
    }
    __syncthreads();
    // step 3: column tile `wave` of the OT row tiles outside the pivot block
    const int c0 = 16 * wave;
    const bool pcol = c0 >= kb && c0 < kb + KB;
    dev::d4 acc3[OT];
#pragma unroll
    for (int s = 0; s < OT; ++s) {
      const int r0 = bj_outside<KB>(s, kb);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc3[s][i] = pcol ? 0.0 : sh.a[(r0 + q + 4 * i) * kBjLd + c0 + m];
    }
#pragma unroll
    for (int kk = 0; kk < KB; kk += 4) {
      const double bv = sh.a[(kb + kk + q) * kBjLd + c0 + m];
#pragma unroll
      for (int s = 0; s < OT; ++s) {
        const double av = sh.a[(bj_outside<KB>(s, kb) + m) * kBjLd + kb + kk + q];
        acc3[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(-av, bv, acc3[s], 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < OT; ++s) {
      const int r0 = bj_outside<KB>(s, kb);
#pragma unroll
      for (int i = 0; i < 4; ++i) sh.a[(r0 + q + 4 * i) * kBjLd + c0 + m] = acc3[s][i];
    }
    __syncthreads();
  }
  bool fin = true;
  {
    const int c = t & (NB - 1);
#pragma unroll 8
    for (int r = t >> 7; r < NB; r += kBjThreads / NB) {
      const double v = sh.a[r * kBjLd + c];
      fin = fin && isfinite(v);
      Dinv[r * NB + c] = v;
    }
  }
  if (!fin) atomicMin(info, k0 + 1);
}

// Launch of the diagonal inverse: GELIM_GJ_TR = 4 (default: 512 threads, two
// waves per SIMD), 8 (256 threads) or 2 (1024 threads: 2048 1.52 ms, slower).  With the padded LDS chunks 4 x 8 tiles
// are the faster shape (hip-rbt factor 2048 1.43 vs 1.52 ms, 4096 3.85 vs
// 4.00, 8192 12.94 vs 13.07; before the padding 8 x 8 was, 1.64 vs 1.73).
// Reserving the inverse's CU (LDS-exclusive launch, no GEMM workgroup beside
// it) changed nothing measurable (profiles/rbt_engine_round3.txt).
// The inverse of the NB x NB block at Ablk; `col` (its first global column)
// only labels a non-finite result in info.
int block_inv(const double* Ablk, int64_t lda, int64_t col, double* Di, int* info, hipStream_t s) {
  // GELIM_GJ_BLOCKED: 1 = the blocked MFMA form with 32-pivot blocks, 2 = with
  // 16-pivot blocks (read per launch)
  const char* eb = std::getenv("GELIM_GJ_BLOCKED");
  const int bj = eb ? std::atoi(eb) : 0;
  if (bj == 1 || bj == 2) {
    if (bj == 1) hipLaunchKernelGGL(bj_inv_kernel<32>, dim3(1), dim3(kBjThreads), 0, s, Ablk, lda, (int)col, Di, info);
    else hipLaunchKernelGGL(bj_inv_kernel<16>, dim3(1), dim3(kBjThreads), 0, s, Ablk, lda, (int)col, Di, info);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  const char* e = std::getenv("GELIM_GJ_TR");  // read per launch (tests switch it)
  const int tr = e && (std::atoi(e) == 8 || std::atoi(e) == 2) ? std::atoi(e) : 4;
  // two Gauss-Jordan steps per barrier (bit-identical): 57.0 vs 58.6 us per
  // block alone (profiles/gj_pair_r4.txt); GELIM_GJ_PAIR=0 for one per barrier
  const char* ep = std::getenv("GELIM_GJ_PAIR");
  if ((tr == 4 || tr == 2) && !(ep && std::atoi(ep) == 0)) {
    if (tr == 4)
      hipLaunchKernelGGL((diag_inv_pair_kernel<4>), dim3(1), dim3(16 * NB / 4), 0, s, Ablk, lda, (int)col, Di, info);
    else
      hipLaunchKernelGGL((diag_inv_pair_kernel<2>), dim3(1), dim3(16 * NB / 2), 0, s, Ablk, lda, (int)col, Di, info);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  if (tr == 2)
    hipLaunchKernelGGL((diag_inv_kernel<double, 2>), dim3(1), dim3(16 * NB / 2), 0, s, Ablk, lda, (int)col, Di,
                       (double*)nullptr, info);
  else if (tr == 4)
    hipLaunchKernelGGL((diag_inv_kernel<double, 4>), dim3(1), dim3(16 * NB / 4), 0, s, Ablk, lda, (int)col, Di,
                       (double*)nullptr, info);
  else
    hipLaunchKernelGGL((diag_inv_kernel<double, 8>), dim3(1), dim3(16 * NB / 8), 0, s, Ablk, lda, (int)col, Di,
                       (double*)nullptr, info);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Diagonal block k0 of the np x np matrix M.
int diag_inv(double* M, int64_t ldm, int64_t k0, double* Di, int* info, hipStream_t s) {
  return block_inv(M + k0 * ldm + k0, ldm, k0, Di, info, s);
}

// ---- persistent block triangular solves ----------------------------------------

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ double bcast_lane(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), l) << 32) |
                                        (unsigned)__builtin_amdgcn_readlane((int)b, l));
}

// x = F^-1 c for the block-unit-lower (UPPER = false) or block-upper (UPPER =
// true) part of the block-LDU factor F (np x np, ldf), with the diagonal
// blocks' inverses Dinv (nblk x NB x NB fp64, row-major).  Workgroup w handles
// block row b = w (lower) or nblk - 1 - w (upper): chain position w, so the
// first block of the chain is the first workgroup dispatched.  Thread (r, q):
// equation 128 b + r, columns 32 q .. 32 q + 31 of every 128-column block.
//
// Hand-off: x is pre-filled with kSentinel (a signalling NaN no arithmetic
// produces); a producer stores its 128 values with agent-scope stores and is
// done, a consumer's lanes load the 32 values of their quarter and spin until
// none is the sentinel -- one store + one load per hand-off, where a flag
// needed store + drain + barrier + flag store + flag poll + value load.
constexpr uint64_t kSentinel = 0x7ff4dead0badf00dull;
constexpr int kXcdSlots = 32;  // packed chain: positions per XCD (one workgroup per CU)

template <typename T>
__device__ __forceinline__ void load_blk(T (&u)[kQW], const T* __restrict__ p) {
#pragma unroll
  for (int j = 0; j < kQW; ++j) u[j] = p[j];
}

// Lanes 0..31 of the calling wave poll the published values x[idx + lane]
// in two parts: issue_x sends the first load, settle_x spins until none is
// the sentinel (lanes 32..63 return 0).  The next block's factor loads are
// issued BETWEEN the two, so the first wait is vmcnt(#factor loads): VMEM
// loads return in order, and a value load issued after the prefetch would
// drain it (one HBM latency per block for a workgroup catching up on many
// already-solved blocks).  settle_x returns false (wave-uniform) when the
// bounded spin expired or another workgroup reported an error.
__device__ __forceinline__ unsigned long long issue_x(const double* __restrict__ x, int idx) {
  const int lane = __lane_id();
  const unsigned long long* p = reinterpret_cast<const unsigned long long*>(x + idx + (lane & (kQW - 1)));
  const unsigned long long v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_sched_barrier(0);  // keep the prefetch that follows after this load
  return v;
}

__device__ __forceinline__ bool settle_x(const double* __restrict__ x, int idx, unsigned long long v, int* err,
                                         double& out, bool nap) {
  const int lane = __lane_id();
  bool ok = true;
  if (__ballot(lane < kQW && v == kSentinel) != 0) {
    const unsigned long long* p = reinterpret_cast<const unsigned long long*>(x + idx + (lane & (kQW - 1)));
    const unsigned long long t0 = rtc();
    while (__ballot(lane < kQW && v == kSentinel) != 0) {
      // workgroups further down the chain back off: every waiting wave polls
      // the same two cache lines, and only the next block's owner is urgent
      if (nap) __builtin_amdgcn_s_sleep(2);
      if (lane < kQW && v == kSentinel) v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rtc() - t0 > kSpinTicks || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        if (lane == 0) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  out = lane < kQW ? __builtin_bit_cast(double, v) : 0.0;
  return ok;
}

template <typename T, bool UPPER>
__global__ __launch_bounds__(kDT) void blk_trsv_kernel(const T* __restrict__ F, int64_t ldf,
                                                      const double* __restrict__ Dinv, const double* __restrict__ c,
                                                      double* __restrict__ x, double* __restrict__ ysave, int nblk,
                                                      int* __restrict__ err, unsigned long long* __restrict__ stamps,
                                                      int packed) {
  __shared__ double part[4][NB];
  __shared__ double rb[NB];
  __shared__ int bad;
  const int t = threadIdx.x, r = t & (NB - 1), lane = t & 63;
  const int q = __builtin_amdgcn_readfirstlane(t >> 7);
  // chain position: packed = consecutive positions on one XCD (workgroup ids
  // are dealt to the 8 XCDs round-robin, so id = 8 slot + xcd; position =
  // 32 xcd + slot), keeping most hand-offs inside one XCD's L2; the grid then
  // has 8 * 32 workgroups and the unused ones return at once
  int w = blockIdx.x;
  if (packed) {
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    if (slot >= kXcdSlots) return;
    w = xcd * kXcdSlots + slot;
  }
  if (w >= nblk) return;
  const int b = UPPER ? nblk - 1 - w : w;
  const int row = NB * b + r;
  if (t == 0) bad = 0;
  // this block's inverse row and right-hand side (independent of
  // everything): loaded first and pinned in registers here -- left to the
  // scheduler, the loads sank past the block loop and their HBM latency
  // (2-5 us at 8192) landed on the chain, between the last hand-off and the
  // publish (scripts/trsv_stamps.py)
  double dv[kQW];
  {
    const double* d = Dinv + ((int64_t)b * NB + r) * NB + kQW * q;
#pragma unroll
    for (int j = 0; j < kQW; ++j) dv[j] = d[j];
  }
  double cv = c[row];
#pragma unroll
  for (int j = 0; j < kQW; ++j) asm volatile("" : "+v"(dv[j]));
  asm volatile("" : "+v"(cv));
  if (stamps && t == 0) stamps[3 * w] = rtc();
  double acc = 0.0;
  const T* frow = F + (int64_t)row * ldf + kQW * q;
  auto blk = [&](int i) { return frow + (int64_t)NB * (UPPER ? nblk - 1 - i : i); };
  auto xidx = [&](int i) { return NB * (UPPER ? nblk - 1 - i : i) + kQW * q; };
  bool ok = true;
  T ua[kQW], ub[kQW];
  auto step = [&](const T(&u)[kQW], unsigned long long v, int i) -> bool {
    double xl;
    if (!settle_x(x, xidx(i), v, err, xl, i + 1 < w)) return false;
#pragma unroll
    for (int j = 0; j < kQW; ++j) acc = fma(-(double)u[j], bcast_lane(xl, j), acc);
    return true;
  };
  // Two passes over ONE copy of the finish code: pass 0 runs it on zeros
  // before the block loop (no stores), so its instructions are in the
  // instruction cache when the real finish -- the chain's critical section,
  // executed once per workgroup -- runs in pass 1 (cold, it took 3 us even
  // for block 0, which has no predecessor: scripts/trsv_stamps.py).
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1) {
      if (w > 0) load_blk(ua, blk(0));
      int i = 0;
      // pairs of blocks with the next block's factor loads issued between the
      // values' first load and their wait (straight-line: the wait counts
      // them); no prefetch past the last block -- a load still in flight at
      // the end would hold its registers, and the finish would wait for it
      for (; i + 2 < w; i += 2) {
        unsigned long long v = issue_x(x, xidx(i));
        load_blk(ub, blk(i + 1));
        if (!step(ua, v, i)) { ok = false; break; }
        v = issue_x(x, xidx(i + 1));
        load_blk(ua, blk(i + 2));
        if (!step(ub, v, i + 1)) { ok = false; break; }
      }
      if (ok && i + 1 < w) {  // two blocks left
        unsigned long long v = issue_x(x, xidx(i));
        load_blk(ub, blk(i + 1));
        ok = step(ua, v, i);
        if (ok) ok = step(ub, issue_x(x, xidx(i + 1)), i + 1);
      } else if (ok && i < w) {  // one block left
        ok = step(ua, issue_x(x, xidx(i)), i);
      }
      if (stamps && t == 0) stamps[3 * w + 1] = rtc();  // wave 0 has its last block's values
    }
    const bool real = pass == 1;
    part[q][r] = acc;
    if (!ok && lane == 0) bad = 1;
    __syncthreads();
    if (bad) return;  // uniform: a timed-out wave makes the whole workgroup stop
    if (q == 0) {
      const double y = cv + part[0][r] + part[1][r] + part[2][r] + part[3][r];
      rb[r] = y;
      if (real && ysave) ysave[row] = y;
    }
    __syncthreads();
    double xs = 0.0;
#pragma unroll
    for (int j = 0; j < kQW; ++j) xs = fma(dv[j], rb[kQW * q + j], xs);
    __syncthreads();  // everyone has read rb / part
    part[q][r] = xs;
    __syncthreads();
    if (q == 0 && real) {
      double xv = part[0][r] + part[1][r] + part[2][r] + part[3][r];
      if (__builtin_bit_cast(unsigned long long, xv) == kSentinel) xv = __builtin_nan("");  // never publish the sentinel
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + row), __builtin_bit_cast(unsigned long long, xv),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (stamps && t == 0) stamps[3 * w + 2] = rtc();
    }
    __syncthreads();  // pass 0's reads of part are done before pass 1 writes it
  }
}

__global__ __launch_bounds__(256) void fill_sentinel_kernel(unsigned long long* __restrict__ p, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = kSentinel;
}

// One launch before both triangular solves: both hand-off buffers (forward
// z, backward x; x must not alias the forward's input) sentinel-filled.
__global__ __launch_bounds__(256) void prep_solves_kernel(unsigned long long* __restrict__ z,
                                                          unsigned long long* __restrict__ x, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    z[i] = kSentinel;
    x[i] = kSentinel;
  }
}

// omega = max_i |r_i| / w_i (componentwise backward error; w_i = 0 counts as
// 0), one workgroup, written to *out.
__global__ __launch_bounds__(1024) void berr_kernel(const double* __restrict__ r, const double* __restrict__ w, int n,
                                                   double* __restrict__ out) {
  __shared__ double red[16];
  double m = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const double wi = w[i], ri = fabs(r[i]);
    const double v = wi > 0.0 ? ri / wi : (ri > 0.0 ? INFINITY : 0.0);
    m = (v > m || v != v) ? v : m;  // NaN propagates
  }
  m = dev::wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x < 64) {
    double v = threadIdx.x < 16 ? red[threadIdx.x] : 0.0;
    v = dev::wave_max(v);
    if (threadIdx.x == 0) *out = v;
  }
}

__global__ __launch_bounds__(256) void axpy_kernel(double* __restrict__ x, const double* __restrict__ d, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) x[i] += d[i];
}

// Rounded fp32 copy of a rows x cols fp64 block (the fp32 engine's GEMM operands).
__global__ __launch_bounds__(256) void to_f32_kernel(const double* __restrict__ src, int64_t sld,
                                                    float* __restrict__ dst, int64_t dld, int cols) {
  const int64_t r = blockIdx.y;
  for (int c = blockIdx.x * 256 + threadIdx.x; c < cols; c += gridDim.x * 256)
    dst[r * dld + c] = (float)src[r * sld + c];
}

int to_f32(const double* src, int64_t sld, float* dst, int64_t dld, int64_t rows, int64_t cols, hipStream_t s) {
  const unsigned gx = (unsigned)std::min<int64_t>((cols + 255) / 256, 64);
  hipLaunchKernelGGL(to_f32_kernel, dim3(gx, (unsigned)rows), dim3(256), 0, s, src, sld, dst, dld, (int)cols);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Block LDU factorisation of the transformed (fp64) matrix in place: per
// block k, Dinv_k = A_kk^-1 (fp64 Gauss-Jordan), W = A_kk^-1 A_k,rest (fp64
// MFMA), A_rest,rest -= A_rest,k W -- on the fp64 matrix cores, or (A21f /
// Wf given: the fp32 engine) as an fp32 MFMA product of rounded copies
// accumulated into the fp64 matrix.  Only that O(n^3) product is fp32: the
// inverses and W stay fp64, so a badly conditioned diagonal block costs
// cond * eps64, not cond * eps32.
int factor_impl(double* M, int64_t ldm, int64_t np, double* Dinv, double* W, float* A21f, float* Wf, int* info,
                hipStream_t s) {
  for (int64_t k0 = 0; k0 < np; k0 += NB) {
    double* Di = Dinv + (k0 / NB) * NB * NB;
    GELIM_TRY(diag_inv(M, ldm, k0, Di, info, s));
    const int64_t rest = np - k0 - NB;
    if (rest <= 0) break;
    double* A12 = M + k0 * ldm + k0 + NB;
    double* A21 = M + (k0 + NB) * ldm + k0;
    double* A22 = M + (k0 + NB) * ldm + k0 + NB;
    GELIM_TRY(dgemm_ex(W, rest, Di, NB, A12, ldm, NB, rest, NB, 1.0, 0, s));  // W = A11^-1 A12
    if (!A21f) {
      GELIM_TRY(dgemm_ex(A22, ldm, A21, ldm, W, rest, rest, rest, NB, -1.0, 1, s));  // A22 -= A21 W
    } else {
      GELIM_TRY(to_f32(A21, ldm, A21f, NB, rest, NB, s));
      GELIM_TRY(to_f32(W, rest, Wf, rest, NB, rest, s));
      GELIM_TRY(matmul_f32(A21f, NB, Wf, rest, nullptr, ldm, rest, rest, NB, 1, GELIM_MM_MFMA, s, -1.0f, A22));
    }
  }
  return GELIM_OK;
}

// The same factorisation with a one-block lookahead on two streams (fp64):
// after W_k, the main stream updates only block column k+1 and block row k+1
// (two thin GEMMs) and inverts the next diagonal block at once, while the
// side stream runs the big trailing update of step k (rows / columns >= k+2)
// (optionally on a grid capped below the CU count, GELIM_RBT_RESERVE).  Main waits for side step k-1 before touching block row / column
// k+1 (the side's step k-1 region); W is double-buffered (side step k reads
// W_k while main computes W_{k+1}).
int factor_la(double* M, int64_t ldm, int64_t np, double* Dinv, double* W2, int* info, hipStream_t s,
              hipStream_t side, hipEvent_t e0, hipEvent_t e1, int cap) {
  const int64_t nblk = np / NB;
  GELIM_TRY(diag_inv(M, ldm, 0, Dinv, info, s));
  bool side_used = false;
  for (int64_t k = 0; k + 1 < nblk; ++k) {
    const int64_t k0 = k * NB, rest = np - k0 - NB, rest2 = rest - NB;
    double* Di = Dinv + k * NB * NB;
    double* Wk = W2 + (k & 1) * NB * np;
    double* A21 = M + (k0 + NB) * ldm + k0;
    GELIM_TRY(dgemm_ex(Wk, rest, Di, NB, M + k0 * ldm + k0 + NB, ldm, NB, rest, NB, 1.0, 0, s));  // W_k
    if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));  // side step k-1 done
    // block column k+1 (all rows below k), then block row k+1 (columns past k+1)
    GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + NB, ldm, A21, ldm, Wk, rest, rest, NB, NB, -1.0, 1, s));
    if (rest2 > 0) {
      GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + 2 * NB, ldm, A21, ldm, Wk + NB, rest, NB, rest2, NB, -1.0, 1, s));
      HIP_TRY(hipEventRecord(e0, s));
      HIP_TRY(hipStreamWaitEvent(side, e0, 0));
      GELIM_TRY(dgemm_capped(M + (k0 + 2 * NB) * ldm + k0 + 2 * NB, ldm, M + (k0 + 2 * NB) * ldm + k0, ldm, Wk + NB,
                             rest, rest2, rest2, NB, -1.0, cap, side, 1));
      HIP_TRY(hipEventRecord(e1, side));
      side_used = true;
    }
    GELIM_TRY(diag_inv(M, ldm, k0 + NB, Dinv + (k + 1) * NB * NB, info, s));
  }
  if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));
  return GELIM_OK;
}

// Lookahead with PAIRS of blocks per trailing update (fp64): the big update
// runs once per two blocks with K = 256 (dgemm 41-43 TF/s at K = 256 vs ~32
// at K = 128, and half the C traffic), and the main stream works one pair
// ahead of it.  Pair p = blocks (k, k+1), whose block rows / columns are up
// to date when it starts; main stream:
//   W1 = D_k A[k, k+1:]  (rows 0..127 of the pair's W)
//   A[k+1:, k+1] -= A[k+1:, k] W1[:, k+1];  A[k+1, k+2:] -= A[k+1, k] W1[:, k+2:]
//   D_{k+1};  W2 = D_{k+1} A[k+1, k+2:]  (rows 128..255, column offset 128)
//   [wait: side's update of pair p-1]
//   next pair's panel (block columns k+2, k+3, all rows below; then their block
//   rows right of them): -= A[., k:k+2] [W1; W2] (K = 256)
//   D_{k+2}, and on to pair p+1 -- while the side stream runs
//   A[k+4:, k+4:] -= A[k+4:, k:k+2] [W1; W2][:, k+4:]  (K = 256).
// The pair's W is double-buffered (side reads pair p while main builds p+1).
int factor_la2(double* M, int64_t ldm, int64_t np, double* Dinv, double* W4, int* info, hipStream_t s,
               hipStream_t side, hipEvent_t e0, hipEvent_t e1, int cap) {
  const int64_t nblk = np / NB;
  GELIM_TRY(diag_inv(M, ldm, 0, Dinv, info, s));
  bool side_used = false;
  for (int64_t k = 0, pair = 0; k + 1 < nblk; k += 2, ++pair) {
    const int64_t k0 = k * NB, r1 = np - k0 - NB;  // columns right of block k
    double* Wp = W4 + (pair & 1) * 2 * NB * np;    // 2 NB rows, ld r1
    double* Ak = M + (k0 + NB) * ldm + k0;         // A[k+1:, k]
    GELIM_TRY(dgemm_ex(Wp, r1, Dinv + k * NB * NB, NB, M + k0 * ldm + k0 + NB, ldm, NB, r1, NB, 1.0, 0, s));
    // step k on block k+1: its column (rows k+1..), its row (columns k+2..)
    GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + NB, ldm, Ak, ldm, Wp, r1, r1, NB, NB, -1.0, 1, s));
    const int64_t r2 = r1 - NB;  // columns right of block k+1
    if (r2 > 0)
      GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + 2 * NB, ldm, Ak, ldm, Wp + NB, r1, NB, r2, NB, -1.0, 1, s));
    GELIM_TRY(diag_inv(M, ldm, k0 + NB, Dinv + (k + 1) * NB * NB, info, s));
    if (r2 <= 0) break;  // block k+1 was the last
    GELIM_TRY(dgemm_ex(Wp + NB * r1 + NB, r1, Dinv + (k + 1) * NB * NB, NB, M + (k0 + NB) * ldm + k0 + 2 * NB, ldm,
                       NB, r2, NB, 1.0, 0, s));
    if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));  // side's pair p-1 update (rows / columns >= k+2)
    // the next pair's panel: block columns k+2 .. k+2+pw (all rows >= k+2),
    // then its block rows right of it
    const int64_t pw = std::min<int64_t>(2 * NB, r2);   // panel width
    const int64_t r4 = r2 - pw;                        // columns right of the panel
    double* A2 = M + (k0 + 2 * NB) * ldm + k0;         // A[k+2:, k:k+2]
    GELIM_TRY(dgemm_ex(M + (k0 + 2 * NB) * ldm + k0 + 2 * NB, ldm, A2, ldm, Wp + NB, r1, r2, pw, 2 * NB, -1.0, 1, s));
    if (r4 > 0) {
      GELIM_TRY(dgemm_ex(M + (k0 + 2 * NB) * ldm + k0 + 2 * NB + pw, ldm, A2, ldm, Wp + NB + pw, r1, pw, r4, 2 * NB,
                         -1.0, 1, s));
      HIP_TRY(hipEventRecord(e0, s));
      HIP_TRY(hipStreamWaitEvent(side, e0, 0));
      GELIM_TRY(dgemm_capped(M + (k0 + 2 * NB + pw) * ldm + k0 + 2 * NB + pw, ldm, M + (k0 + 2 * NB + pw) * ldm + k0,
                             ldm, Wp + NB + pw, r1, r4, r4, 2 * NB, -1.0, cap, side, 1));
      HIP_TRY(hipEventRecord(e1, side));
      side_used = true;
    }
    GELIM_TRY(diag_inv(M, ldm, k0 + 2 * NB, Dinv + (k + 2) * NB * NB, info, s));
  }
  if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));
  return GELIM_OK;
}

// factor_la2 with a third stream (aux) that takes every update the next
// diagonal inverse does not read, so it runs UNDER that inverse (a one-
// workgroup kernel) instead of before it.  Per pair (k, k+1):
//   main: W1 = D_k A[k, k+1:];  A[k+1, k+1] -= A[k+1, k] W1[:, :128]   (diagonal block only)
//   aux:  A[k+2:, k+1] -= A[k+2:, k] W1[:, :128];  A[k+1, k+2:] -= A[k+1, k] W1[:, 128:]
//   main: D_{k+1}; [join aux]; W2 = D_{k+1} A[k+1, k+2:]; [wait side p-1; side p may start]
//   main: panel rows k+2 only: A[k+2, panel] -= A[k+2, k:k+2] [W1; W2][:, panel]
//   aux:  panel rows k+3..:   A[k+3:, panel] -= ...;  panel's block rows right of it (K = 256)
//   main: D_{k+2}; [join aux before the next pair]
// Measured slower than factor_la2 (4096: 4.10 vs 3.96 ms, 8192: 13.64 vs
// 13.07 ms; forced at 2048: 1.73 vs 1.51 ms without lookahead): the inverse
// does not speed up by having the GEMMs beside it, and each pair adds four
// cross-stream event waits.  Off by default (GELIM_RBT_AUX=1).
// Regions: aux writes column k+1 below block k+1, row k+1 right of it, the
// panel below its first block row and the panel's block rows right of the
// panel; the side (after the wait on pair p-1) writes rows and columns past
// the panel; main writes only what the next inverse reads.  Every region a
// stream reads was written before the event it waited on.
int factor_la3(double* M, int64_t ldm, int64_t np, double* Dinv, double* W4, int* info, hipStream_t s,
               hipStream_t side, hipStream_t aux, hipEvent_t e0, hipEvent_t e1, hipEvent_t ea, hipEvent_t eb,
               int cap) {
  const int64_t nblk = np / NB;
  GELIM_TRY(diag_inv(M, ldm, 0, Dinv, info, s));
  bool side_used = false, aux_used = false;
  auto fork = [&]() -> int {  // aux continues after everything main issued so far
    HIP_TRY(hipEventRecord(ea, s));
    HIP_TRY(hipStreamWaitEvent(aux, ea, 0));
    return GELIM_OK;
  };
  auto join = [&]() -> int {  // main continues after everything aux issued so far
    if (!aux_used) return GELIM_OK;
    HIP_TRY(hipEventRecord(eb, aux));
    HIP_TRY(hipStreamWaitEvent(s, eb, 0));
    aux_used = false;
    return GELIM_OK;
  };
  for (int64_t k = 0, pair = 0; k + 1 < nblk; k += 2, ++pair) {
    GELIM_TRY(join());  // the previous pair's panel below its first block row / block rows right of it
    const int64_t k0 = k * NB, r1 = np - k0 - NB, r2 = r1 - NB;
    double* Wp = W4 + (pair & 1) * 2 * NB * np;  // 2 NB rows, ld r1
    double* Ak = M + (k0 + NB) * ldm + k0;       // A[k+1:, k]
    GELIM_TRY(dgemm_ex(Wp, r1, Dinv + k * NB * NB, NB, M + k0 * ldm + k0 + NB, ldm, NB, r1, NB, 1.0, 0, s));
    GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + NB, ldm, Ak, ldm, Wp, r1, NB, NB, NB, -1.0, 1, s));
    if (r2 > 0) {
      GELIM_TRY(fork());
      GELIM_TRY(dgemm_ex(M + (k0 + 2 * NB) * ldm + k0 + NB, ldm, Ak + NB * ldm, ldm, Wp, r1, r2, NB, NB, -1.0, 1, aux));
      GELIM_TRY(dgemm_ex(M + (k0 + NB) * ldm + k0 + 2 * NB, ldm, Ak, ldm, Wp + NB, r1, NB, r2, NB, -1.0, 1, aux));
      aux_used = true;
    }
    GELIM_TRY(diag_inv(M, ldm, k0 + NB, Dinv + (k + 1) * NB * NB, info, s));
    if (r2 <= 0) break;  // block k+1 was the last
    GELIM_TRY(join());
    GELIM_TRY(dgemm_ex(Wp + NB * r1 + NB, r1, Dinv + (k + 1) * NB * NB, NB, M + (k0 + NB) * ldm + k0 + 2 * NB, ldm,
                       NB, r2, NB, 1.0, 0, s));
    if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));  // side's pair p-1 update (rows / columns >= k+2)
    const int64_t pw = std::min<int64_t>(2 * NB, r2);  // panel width
    const int64_t r4 = r2 - pw;                       // columns right of the panel
    double* A2 = M + (k0 + 2 * NB) * ldm + k0;        // A[k+2:, k:k+2]
    double* P = M + (k0 + 2 * NB) * ldm + k0 + 2 * NB;  // the panel's first element
    if (r4 > 0) {
      // the side's region (rows / columns past the panel) reads only the
      // final L columns k, k+1 and this pair's W
      HIP_TRY(hipEventRecord(e0, s));
      HIP_TRY(hipStreamWaitEvent(side, e0, 0));
      GELIM_TRY(dgemm_capped(M + (k0 + 2 * NB + pw) * ldm + k0 + 2 * NB + pw, ldm, M + (k0 + 2 * NB + pw) * ldm + k0,
                             ldm, Wp + NB + pw, r1, r4, r4, 2 * NB, -1.0, cap, side, 1));
      HIP_TRY(hipEventRecord(e1, side));
      side_used = true;
    }
    GELIM_TRY(dgemm_ex(P, ldm, A2, ldm, Wp + NB, r1, NB, pw, 2 * NB, -1.0, 1, s));  // block row k+2 of the panel
    if (r2 > NB || r4 > 0) {
      GELIM_TRY(fork());
      if (r2 > NB)
        GELIM_TRY(dgemm_ex(P + NB * ldm, ldm, A2 + NB * ldm, ldm, Wp + NB, r1, r2 - NB, pw, 2 * NB, -1.0, 1, aux));
      if (r4 > 0)
        GELIM_TRY(dgemm_ex(P + pw, ldm, A2, ldm, Wp + NB + pw, r1, pw, r4, 2 * NB, -1.0, 1, aux));
      aux_used = true;
    }
    GELIM_TRY(diag_inv(M, ldm, k0 + 2 * NB, Dinv + (k + 2) * NB * NB, info, s));
  }
  GELIM_TRY(join());
  if (side_used) HIP_TRY(hipStreamWaitEvent(s, e1, 0));
  return GELIM_OK;
}

// Block-LDU solve: forward z_k = D_k^-1 (c_k - sum_{j<k} A_kj z_j) keeping
// y_k = c_k - sum (the block-unit-lower solve's result), then backward
// x_k = D_k^-1 (y_k - sum_{j>k} A_kj x_j).  c -> (z, y) -> x (x may alias c:
// it is sentinel-filled only after the forward solve has read c).
unsigned long long* g_trsv_stamps = nullptr;  // diagnostics: 3 realtime stamps per workgroup (lower solve)

// Returns GELIM_OK, kNotResident (a positive code: the caller falls back to
// partial pivoting) when the persistent grid cannot be co-resident, or < 0.
// The error word flags[0] is NOT cleared here: the caller zeroes it once per
// outer solve (gelim_mixed_reset_error), so a hand-off timeout of any inner
// apply stays visible until it is checked.
constexpr int kNotResident = 1;

template <typename T>
int solve_impl(const T* M, int64_t ldm, int64_t np, const double* Dinv, const double* c, double* z, double* y,
               double* x, unsigned* flags, hipStream_t s) {
  const int nblk = (int)(np / NB);
  static const bool fits = [] {
    int a = 0, b = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, blk_trsv_kernel<T, false>, kDT, 0) == hipSuccess &&
           hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, blk_trsv_kernel<T, true>, kDT, 0) == hipSuccess &&
           a >= 1 && b >= 1;
  }();
  static const int pack_env = [] {
    const char* e = std::getenv("GELIM_TRSV_PACK");
    return e ? std::atoi(e) : 1;
  }();
  // the XCD-packed chain maps positions across the whole 8 x 32 grid (position
  // 32 is workgroup 1, waiting on position 31 = workgroup 248), so it needs
  // every one of them resident; one workgroup per block row needs only nblk
  // (workgroups are dispatched in order, each waits on lower ids only)
  if (!fits || nblk > kMaxBlocks) return kNotResident;
  const int pack = pack_env && coresident(1, 8 * kXcdSlots) ? 1 : 0;
  if (!pack && !coresident(1, nblk)) return kNotResident;
  int* err = reinterpret_cast<int*>(flags);  // flags[0]: error word
  const unsigned g = (unsigned)((np + 255) / 256);
  const bool alias = x == c;  // x is then sentinel-filled only after the forward solve has read c
  if (alias) {
    hipLaunchKernelGGL(fill_sentinel_kernel, dim3(g), dim3(256), 0, s, reinterpret_cast<unsigned long long*>(z),
                       (int)np);
  } else {
    hipLaunchKernelGGL(prep_solves_kernel, dim3(g), dim3(256), 0, s, reinterpret_cast<unsigned long long*>(z),
                       reinterpret_cast<unsigned long long*>(x), (int)np);
  }
  HIP_TRY(hipGetLastError());
  const unsigned grid = pack ? 8u * kXcdSlots : (unsigned)nblk;
  hipLaunchKernelGGL((blk_trsv_kernel<T, false>), dim3(grid), dim3(kDT), 0, s, M, ldm, Dinv, c, z, y, nblk, err,
                     g_trsv_stamps, pack);
  HIP_TRY(hipGetLastError());
  if (alias) {
    hipLaunchKernelGGL(fill_sentinel_kernel, dim3(g), dim3(256), 0, s, reinterpret_cast<unsigned long long*>(x),
                       (int)np);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL((blk_trsv_kernel<T, true>), dim3(grid), dim3(kDT), 0, s, M, ldm, Dinv, y, x, (double*)nullptr,
                     nblk, err, (unsigned long long*)nullptr, pack);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace
}  // namespace gelim

struct gelim_mixed_plan {
  int64_t n = 0, np = 0, ldm = 0;
  int fp64 = 0;             // factor precision: 0 fp32 ("hip-mixed"), 1 fp64 ("hip-rbt")
  double* M = nullptr;      // np x ldm: the transformed matrix, then its block-LDU factor
  double* Dinv = nullptr;   // nblk x NB x NB: inverse of every (Schur) diagonal block
  double* W = nullptr;      // 4 x NB x np: A_kk^-1 A_k,rest (pairs of blocks, double-buffered under lookahead)
  float* A21f = nullptr;    // np x NB, NB x np: rounded GEMM operands (fp32 engine only)
  float* Wf = nullptr;
  double* ud = nullptr;     // U's butterfly diagonals (8 x np/4)
  double* vd = nullptr;     // V's
  unsigned* flags = nullptr;  // [0]: the solves' error word
  double* c = nullptr;      // U^T r (np)
  double* y = nullptr;      // L^-1 c (np)
  double* z = nullptr;      // U^-1 y (np)
  double* xs = nullptr;     // the backward solve's hand-off buffer (np): filled with z before the forward solve
  int* info = nullptr;
  int err_host = 0;
  double* rv = nullptr;     // refinement (gelim_mixed_solve): r, |b| + |A||x|, correction, best x (n each)
  double* wv = nullptr;
  double* dv = nullptr;
  double* xb = nullptr;
  double* om = nullptr;     // device scalar: the backward error
  int lookahead = 0;        // fp64 engine: lookahead on a side stream
  int pairs = 1;            // lookahead over pairs of blocks (K = 256 trailing updates)
  int cap = 0;              // side-stream GEMM grid cap (CUs)
  hipStream_t side = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int aux_on = 0;              // pairs: updates the next inverse does not read on a third stream (factor_la3)
  hipStream_t aux = nullptr;
  hipEvent_t ea = nullptr, eb = nullptr;
  hipStream_t crit = nullptr;  // GELIM_CRIT_PRIO set: the factorisation's chain on a stream of that priority
  hipEvent_t ef = nullptr, ej = nullptr;
};

extern "C" int64_t gelim_mixed_max_n(void) { return (int64_t)gelim::kMaxBlocks * gelim::NB; }

extern "C" void gelim_mixed_plan_destroy(gelim_mixed_plan* p) {
  if (!p) return;
  for (void* q : {(void*)p->M, (void*)p->Dinv, (void*)p->W, (void*)p->A21f, (void*)p->Wf, (void*)p->ud, (void*)p->vd,
                  (void*)p->rv, (void*)p->wv, (void*)p->dv, (void*)p->xb, (void*)p->om, (void*)p->flags, (void*)p->c,
                  (void*)p->y, (void*)p->z, (void*)p->xs, (void*)p->info})
    (void)hipFree(q);
  if (p->ea) (void)hipEventDestroy(p->ea);
  if (p->eb) (void)hipEventDestroy(p->eb);
  if (p->aux) (void)hipStreamDestroy(p->aux);
  if (p->e0) (void)hipEventDestroy(p->e0);
  if (p->e1) (void)hipEventDestroy(p->e1);
  if (p->side) (void)hipStreamDestroy(p->side);
  if (p->ef) (void)hipEventDestroy(p->ef);
  if (p->ej) (void)hipEventDestroy(p->ej);
  if (p->crit) (void)hipStreamDestroy(p->crit);
  delete p;
}

// n: order of the system; ud / vd: host arrays of 8 * np/4 butterfly entries
// each (np = gelim_mixed_padded(n)), exp(r/10) with r uniform in [-1/2, 1/2].
extern "C" int64_t gelim_mixed_padded(int64_t n) { return (n + gelim::kPadTo - 1) / gelim::kPadTo * gelim::kPadTo; }

// fp64 = 0: fp32 factors (GMRES-IR in the caller), 1: fp64 factors.
extern "C" gelim_mixed_plan* gelim_mixed_plan_create2(int64_t n, const double* ud, const double* vd, int fp64) {
  const int64_t np = gelim_mixed_padded(n);
  if (n <= 0 || np > gelim_mixed_max_n()) {
    GELIM_FAIL(GELIM_E_ARG, "mixed plan: n must be in [1, " + std::to_string(gelim_mixed_max_n()) +
                                "] (persistent triangular solves: every 128-row block resident)");
    return nullptr;
  }
  auto* p = new gelim_mixed_plan;
  p->n = n;
  p->np = np;
  p->fp64 = fp64 ? 1 : 0;
  p->ldm = np + 2;  // 16-byte rows, off the power-of-two stride
  auto fail = [&](const char* what) -> gelim_mixed_plan* {
    GELIM_FAIL(GELIM_E_NOMEM, std::string("mixed plan: ") + what);
    gelim_mixed_plan_destroy(p);
    return nullptr;
  };
  const size_t nd = (size_t)2 * np;  // 8 arrays of np/4
  const int64_t nblk = np / gelim::NB;
  if (hipMalloc((void**)&p->M, sizeof(double) * (size_t)np * p->ldm) != hipSuccess) return fail("matrix");
  if (hipMalloc((void**)&p->Dinv, sizeof(double) * (size_t)np * gelim::NB) != hipSuccess) return fail("inverses");
  if (hipMalloc((void**)&p->W, 4 * sizeof(double) * (size_t)np * gelim::NB) != hipSuccess) return fail("W buffer");
  // lookahead (fp64): from 32 blocks (n = 4096) unless GELIM_RBT_LOOKAHEAD says otherwise
  {
    const char* e = std::getenv("GELIM_RBT_LOOKAHEAD");
    p->lookahead = fp64 && (e ? std::atoi(e) != 0 : np >= 4096);
    const char* ep = std::getenv("GELIM_RBT_PAIRS");
    p->pairs = ep ? std::atoi(ep) != 0 : 1;
    const char* ex = std::getenv("GELIM_RBT_AUX");
    p->aux_on = ex ? std::atoi(ex) != 0 : 0;  // measured slower (profiles/rbt_engine_round3.txt)
  }
  if (p->lookahead) {
    int dev = 0, ncu = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    // side grid: uncapped by default (the regular dgemm kernel; the one-CU
    // inverse still gets a CU as the GEMM's short-lived workgroups retire):
    // 8192 15.0 ms, 16384 87.6 ms vs 18.7 / 122.7 ms with the persistent
    // kernel capped 64 CUs short, and 16.0 / 91.3 ms without lookahead
    int reserve = 0;
    if (const char* e = std::getenv("GELIM_RBT_RESERVE")) reserve = std::max(0, std::atoi(e));
    p->cap = reserve == 0 ? 0 : ncu > reserve + 8 ? ncu - reserve : std::max(8, ncu / 2);
    // GELIM_RBT_MASK=<k>: the side stream's GEMMs stay off k CUs (CU-masked
    // queue; GELIM_RBT_MASK_SPREAD=0 takes the lowest-numbered CUs) and the
    // chain runs on a stream of its own, so its thin GEMMs and inverses
    // always find free CUs
    int mask = 0, spread = 1;
    if (const char* e = std::getenv("GELIM_RBT_MASK")) mask = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GELIM_RBT_MASK_SPREAD")) spread = std::atoi(e) != 0;
    if (mask > 0) {
      if (gelim::masked_stream_create(&p->side, mask, spread) != GELIM_OK) return fail("masked side stream");
    } else if (gelim::side_stream_create(&p->side) != GELIM_OK) {
      return fail("side stream");
    }
    if (mask > 0 || std::getenv("GELIM_CRIT_PRIO")) {
      const char* ec = std::getenv("GELIM_RBT_MASK_CRIT");  // 1: the chain on the reserved CUs alone
      if (mask > 0 && ec && std::atoi(ec) != 0) {
        if (gelim::masked_stream_create(&p->crit, mask, spread, true) != GELIM_OK) return fail("critical stream");
      } else if (gelim::side_stream_create(&p->crit, 1) != GELIM_OK) {
        return fail("critical stream");
      }
      if (hipEventCreateWithFlags(&p->ef, hipEventDisableTiming) != hipSuccess) return fail("event");
      if (hipEventCreateWithFlags(&p->ej, hipEventDisableTiming) != hipSuccess) return fail("event");
    }
    if (hipEventCreateWithFlags(&p->e0, hipEventDisableTiming) != hipSuccess) return fail("event");
    if (hipEventCreateWithFlags(&p->e1, hipEventDisableTiming) != hipSuccess) return fail("event");
    if (p->pairs && p->aux_on) {
      if (gelim::side_stream_create(&p->aux) != GELIM_OK) return fail("aux stream");
      if (hipEventCreateWithFlags(&p->ea, hipEventDisableTiming) != hipSuccess) return fail("event");
      if (hipEventCreateWithFlags(&p->eb, hipEventDisableTiming) != hipSuccess) return fail("event");
    }
  }
  if (!fp64 && hipMalloc((void**)&p->A21f, sizeof(float) * (size_t)np * gelim::NB) != hipSuccess) return fail("A21f");
  if (!fp64 && hipMalloc((void**)&p->Wf, sizeof(float) * (size_t)np * gelim::NB) != hipSuccess) return fail("Wf");
  if (hipMalloc((void**)&p->ud, sizeof(double) * nd) != hipSuccess) return fail("ud");
  if (hipMalloc((void**)&p->vd, sizeof(double) * nd) != hipSuccess) return fail("vd");
  (void)nblk;
  if (hipMalloc((void**)&p->flags, 16) != hipSuccess) return fail("flags");
  if (hipMalloc((void**)&p->c, sizeof(double) * np) != hipSuccess) return fail("c");
  if (hipMalloc((void**)&p->y, sizeof(double) * np) != hipSuccess) return fail("y");
  if (hipMalloc((void**)&p->z, sizeof(double) * np) != hipSuccess) return fail("z");
  if (hipMalloc((void**)&p->xs, sizeof(double) * np) != hipSuccess) return fail("xs");
  if (hipMalloc((void**)&p->info, 16) != hipSuccess) return fail("info");
  for (double** b : {&p->rv, &p->wv, &p->dv, &p->xb})
    if (hipMalloc((void**)b, sizeof(double) * (size_t)n) != hipSuccess) return fail("refinement vectors");
  if (hipMalloc((void**)&p->om, 16) != hipSuccess) return fail("omega");
  if (hipMemcpy(p->ud, ud, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("ud copy");
  if (hipMemcpy(p->vd, vd, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("vd copy");
  return p;
}

extern "C" gelim_mixed_plan* gelim_mixed_plan_create(int64_t n, const double* ud, const double* vd) {
  return gelim_mixed_plan_create2(n, ud, vd, 0);
}

// Transform the augmented fp64 system's matrix (n x n at aug, leading
// dimension ld) into the plan's matrix and factor it without pivoting.
// Returns 0, or 1 + the first column whose pivot is zero / not finite (the
// caller then falls back to partial pivoting); < 0 on errors.  Synchronises.
extern "C" int gelim_mixed_factor(gelim_mixed_plan* p, const double* aug, int64_t ld, void* stream) {
  using namespace gelim;
  if (!p || !aug) return GELIM_FAIL(GELIM_E_ARG, "mixed_factor: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t np = p->np, h = np / 4, ldm = p->ldm;
  HIP_TRY(hipMemsetAsync(p->info, 0x7f, 4, s));  // INT_MAX-ish: atomicMin keeps the first bad column
  hipStream_t caller = s;
  if (p->crit) {  // fork onto the critical-priority stream; joined below
    HIP_TRY(hipEventRecord(p->ef, s));
    HIP_TRY(hipStreamWaitEvent(p->crit, p->ef, 0));
    s = p->crit;
  }
  const dim3 grid((unsigned)((h + 255) / 256), (unsigned)h);
  hipLaunchKernelGGL(rbt_matrix_kernel<double>, grid, dim3(256), 0, s, aug, ld, (int)p->n, (int)np, p->ud, p->vd,
                     p->M, ldm);
  HIP_TRY(hipGetLastError());
  if (p->lookahead && p->pairs && p->aux)
    GELIM_TRY(factor_la3(p->M, ldm, np, p->Dinv, p->W, p->info, s, p->side, p->aux, p->e0, p->e1, p->ea, p->eb,
                         p->cap));
  else if (p->lookahead && p->pairs)
    GELIM_TRY(factor_la2(p->M, ldm, np, p->Dinv, p->W, p->info, s, p->side, p->e0, p->e1, p->cap));
  else if (p->lookahead)
    GELIM_TRY(factor_la(p->M, ldm, np, p->Dinv, p->W, p->info, s, p->side, p->e0, p->e1, p->cap));
  else
    GELIM_TRY(factor_impl(p->M, ldm, np, p->Dinv, p->W, p->fp64 ? nullptr : p->A21f, p->fp64 ? nullptr : p->Wf,
                          p->info, s));
  if (p->crit) {
    HIP_TRY(hipEventRecord(p->ej, s));
    HIP_TRY(hipStreamWaitEvent(caller, p->ej, 0));
    s = caller;
  }
  int h_info = 0;
  HIP_TRY(hipMemcpyAsync(&h_info, p->info, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return h_info == 0x7f7f7f7f ? 0 : h_info;
}

// d = V (LU)^-1 U^T [r; 0]: the correction of one refinement step (r, d:
// n fp64 entries, r with stride incr).  fp64 arithmetic over the factors.
extern "C" int gelim_mixed_apply(gelim_mixed_plan* p, const double* r, int64_t incr, double* d, void* stream) {
  using namespace gelim;
  if (!p || !r || !d) return GELIM_FAIL(GELIM_E_ARG, "mixed_apply: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int64_t np = p->np, h = np / 4;
  const unsigned g = (unsigned)((h + 255) / 256);
  hipLaunchKernelGGL(rbt_vec_kernel, dim3(g), dim3(256), 0, s, r, incr, (int)p->n, (int)np, p->ud, 1, p->c, (int)np);
  HIP_TRY(hipGetLastError());
  // c -> z (scratch), y (block-unit-lower result) -> xs (the solution of the transformed system)
  const int rc = solve_impl<double>(p->M, p->ldm, np, p->Dinv, p->c, p->z, p->y, p->xs, p->flags, s);
  if (rc != GELIM_OK) return rc;  // < 0: error; kNotResident: the caller falls back
  // x = V xs, only the first n entries are kept (the padding's are zero in exact arithmetic)
  hipLaunchKernelGGL(rbt_vec_kernel, dim3(g), dim3(256), 0, s, p->xs, (int64_t)1, (int)np, (int)np, p->vd, 0, d,
                     (int)p->n);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

extern "C" int gelim_mixed_solve_error(gelim_mixed_plan* p, void* stream);

// Zero the solves' hand-off error word (once per outer solve: every apply of
// that solve then only ever sets it, so one check covers all of them).
extern "C" int gelim_mixed_reset_error(gelim_mixed_plan* p, void* stream) {
  if (!p) return GELIM_FAIL(GELIM_E_ARG, "mixed_reset_error: null plan");
  return gelim::zero_async(p->flags, 16, (hipStream_t)stream);
}

// The whole randomised solve of an augmented fp64 system (n x >= n+1 at aug,
// leading dimension ld) into x (n fp64, device): factorisation, x = (LU)^-1 b,
// then classic fp64 refinement x += (LU)^-1 (b - A x) until the componentwise
// backward error max_i |r_i| / (|b| + |A||x|)_i is <= 4 eps64; once a
// correction stops reducing it by 10 %, or after max_steps corrections, x is
// accepted if it is <= max(sqrt(n), 8) eps64.  Returns 0 (x written; *steps =
// corrections, *berr = final backward error), 1 when the caller must fall
// back to partial pivoting (zero / non-finite pivot or stalled refinement;
// *berr says how far it got), < 0 on errors.  One 8-byte device-to-host read
// per correction (the convergence test); the Python GMRES-IR of the fp32
// engine does not use this.
extern "C" int gelim_mixed_solve(gelim_mixed_plan* p, const double* aug, int64_t ld, double* x, int max_steps,
                                 int* steps, double* berr, void* stream) {
  using namespace gelim;
  if (!p || !aug || !x) return GELIM_FAIL(GELIM_E_ARG, "mixed_solve: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int n = (int)p->n;
  if (steps) *steps = 0;
  if (berr) *berr = INFINITY;
  const int rc = gelim_mixed_factor(p, aug, ld, stream);
  if (rc < 0) return rc;
  if (rc > 0) return 1;
  GELIM_TRY(gelim_mixed_reset_error(p, stream));
  {
    const int ra = gelim_mixed_apply(p, aug + n, ld, x, stream);
    if (ra < 0) return ra;
    if (ra > 0) return 1;  // the persistent solves cannot be resident: partial pivoting instead
  }
  const double eps = 2.220446049250313e-16;
  const double strict = 4.0 * eps, loose = std::max(std::sqrt((double)n), 8.0) * eps;
  double prev = INFINITY, best = INFINITY;
  const unsigned g = (unsigned)((n + 255) / 256);
  for (int it = 0;; ++it) {
    GELIM_TRY(residual_f64(aug, ld, n, x, p->rv, s, 0, p->wv));
    hipLaunchKernelGGL(berr_kernel, dim3(1), dim3(1024), 0, s, p->rv, p->wv, n, p->om);
    HIP_TRY(hipGetLastError());
    double om = 0.0;
    HIP_TRY(hipMemcpyAsync(&om, p->om, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&p->err_host, p->flags, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    // the error word covers every apply since the reset (the first one
    // included): a timed-out hand-off leaves x incomplete -> fall back
    if (p->err_host != 0) {
      if (steps) *steps = it;
      return 1;
    }
    if (steps) *steps = it;
    if (berr) *berr = om;
    if (om <= strict) return 0;
    if (!(om < 0.9 * prev) || it == max_steps) {  // NaN, stagnated or out of steps
      // the better of the current x and the saved best one, if acceptable
      if (om <= best && om <= loose) return 0;
      if (best <= loose) {
        HIP_TRY(hipMemcpyAsync(x, p->xb, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        if (berr) *berr = best;
        return 0;
      }
      return 1;
    }
    if (om < best) {
      best = om;
      HIP_TRY(hipMemcpyAsync(p->xb, x, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    }
    prev = om;
    const int ra = gelim_mixed_apply(p, p->rv, 1, p->dv, stream);
    if (ra < 0) return ra;
    if (ra > 0) return 1;
    hipLaunchKernelGGL(axpy_kernel, dim3(g), dim3(256), 0, s, x, p->dv, n);
    HIP_TRY(hipGetLastError());
  }
}

// Hand-off error word of the last solve (0: fine, 3: a bounded spin expired).
extern "C" int gelim_mixed_solve_error(gelim_mixed_plan* p, void* stream) {
  if (!p) return GELIM_FAIL(GELIM_E_ARG, "mixed_solve_error: null plan");
  hipStream_t s = (hipStream_t)stream;
  const int64_t nblk = p->np / gelim::NB;
  (void)nblk;
  HIP_TRY(hipMemcpyAsync(&p->err_host, p->flags, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  return p->err_host;
}

extern "C" int64_t gelim_mixed_plan_np(const gelim_mixed_plan* p) { return p ? p->np : 0; }

// Diagnostics: realtime stamps (100 MHz) of the NEXT lower block solves, 3 per
// workgroup (start, last block's values in hand, published) into the device
// buffer `stamps` (null: off).
extern "C" void gelim_debug_trsv_stamps(unsigned long long* stamps) { gelim::g_trsv_stamps = stamps; }

// Device pointers of the plan's buffers (tests / debugging): out[0] = factor
// (np x ldm), out[1] = diagonal-block inverses (nblk x 128 x 128 fp64),
// out[2] = the W side buffer; returns ldm.
extern "C" int64_t gelim_mixed_debug_ptrs(gelim_mixed_plan* p, void** out) {
  if (!p || !out) return 0;
  out[0] = p->M;
  out[1] = p->Dinv;
  out[2] = p->W;
  return p->ldm;
}

// Synchronous device-to-device copy of `bytes` (tests: reading the buffers above).
extern "C" int gelim_mixed_debug_copy(void* dst, const void* src, int64_t bytes) {
  HIP_TRY(hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDeviceToDevice));
  return GELIM_OK;
}

// ---- building blocks of the distributed engine (parallel/dist_rbt.py) --------

// Dinv = inverse of the 128 x 128 fp64 block at Ablk (leading dimension lda)
// by the Gauss-Jordan kernel above; *info (device) gets atomicMin'd with
// 1 + col when the result is not finite.
extern "C" int gelim_rbt_block_inverse(const double* Ablk, int64_t lda, int64_t col, double* Dinv, int* info,
                                       void* stream) {
  if (!Ablk || !Dinv || !info || lda < gelim::NB) return GELIM_FAIL(GELIM_E_ARG, "rbt_block_inverse: bad argument");
  return gelim::block_inv(Ablk, lda, col, Dinv, info, (hipStream_t)stream);
}

// x = T^-1 rhs for the block-unit-lower (upper = 0; ysave, may be null,
// gets y_b = rhs_b - sum_{j<b} F_bj x_j) or the block-upper (upper = 1) part
// of an (nblk * 128)-square block-LDU factor F (leading dimension ldf) whose
// diagonal blocks' inverses are Dinv (nblk x 128 x 128): the persistent block
// solve of the randomised engine above (blk_trsv_kernel, one workgroup per
// block row, chain order = dispatch order, so no co-residency is needed).
// The distributed engine's super-block solves (parallel/dist_rbt.py) use it.
// err: a device int, 3 on a hand-off timeout (left as is otherwise).
extern "C" int gelim_rbt_block_solve(const double* F, int64_t ldf, const double* Dinv, int nblk, const double* rhs,
                                     double* x, double* ysave, int upper, int* err, void* stream) {
  using namespace gelim;
  if (!F || !Dinv || !rhs || !x || !err || nblk < 1 || nblk > kMaxBlocks || ldf < (int64_t)nblk * NB || x == rhs)
    return GELIM_FAIL(GELIM_E_ARG, "rbt_block_solve: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int n = nblk * NB;
  hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<unsigned long long*>(x), n);
  if (upper)
    hipLaunchKernelGGL((blk_trsv_kernel<double, true>), dim3((unsigned)nblk), dim3(kDT), 0, s, F, ldf, Dinv, rhs, x,
                       (double*)nullptr, nblk, err, (unsigned long long*)nullptr, 0);
  else
    hipLaunchKernelGGL((blk_trsv_kernel<double, false>), dim3((unsigned)nblk), dim3(kDT), 0, s, F, ldf, Dinv, rhs, x,
                       ysave, nblk, err, (unsigned long long*)nullptr, 0);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// out = U^T [b; 0] (transpose = 1) or out = V y (transpose = 0) for the
// butterfly with diagonals d (8 x np/4, device), b / y of n entries (stride
// incb), out of nout entries -- replicated vectors of the distributed solve.
extern "C" int gelim_rbt_vec(const double* b, int64_t incb, int64_t n, int64_t np, const double* d, int transpose,
                             double* out, int64_t nout, void* stream) {
  if (!b || !d || !out || np % 4 || n > np || nout > np) return GELIM_FAIL(GELIM_E_ARG, "rbt_vec: bad argument");
  const int64_t h = np / 4;
  hipLaunchKernelGGL(gelim::rbt_vec_kernel, dim3((unsigned)((h + 255) / 256)), dim3(256), 0, (hipStream_t)stream, b,
                     incb, (int)n, (int)np, d, transpose, out, (int)nout);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}
