// Randomised no-pivoting engine (GaussSolver backend "hip-rbt"): a random
// butterfly transform (RBT) of the system, a NO-pivoting blocked LU of the
// transformed matrix on the fp64 matrix cores, and fp64 iterative refinement
// against the original system (gelim_mixed_solve; when it does not reach the
// fp64 error class the solver falls back to the partial-pivoting engine).
// (Round 3-4 also had fp32 trailing products + GMRES-IR, "hip-mixed": slower
// than this fp64 engine at every n and not convergent at 16384 -- removed in
// round 5, profiles/trsv_split_r5.txt.)
//
// Factorisation: block LDU without pivoting, 128-column blocks.  Per block k:
//  * diag_inv_pair_kernel: ONE workgroup inverts the (Schur) diagonal block
//    A_kk by Gauss-Jordan in fp64 registers (4 x 8 tiles per thread, uniform
//    rank-1 updates, one barrier per two columns) -> Dinv_k (kept for the solves);
//  * W = A_kk^-1 A_k,rest and A_rest,rest -= A_rest,k W on the matrix cores
//    (dgemm.hip v_mfma_f64_16x16x4f64).  A_rest,k and A_k,rest stay in place
//    as the factor's off-diagonal blocks.
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
// One workgroup of 512 threads (two waves per SIMD) inverts the 128 x 128
// block in place in registers: thread (rg, cg) = (t >> 4, t & 15) holds the
// 4 x 8 tile rows 4 rg.., columns 8 cg...  Step k of Gauss-Jordan is ONE
// rank-1 update of the whole block from a base with row k and column k zeroed,
//   a'[i][j] = b_ij - G_i U_j,  G_i = a[i][k] (G_k = -1),  U_j = a[k][j] / a[k][k] (U_k = 1 / a[k][k]),
// which gives a'[k][k] = 1/a_kk, a'[k][j] = a_kj/a_kk, a'[i][k] = -a_ik/a_kk
// and the Schur update elsewhere with no cancellation (round 6: the earlier
// uniform form a -= g u^T with g_k = a_kk - 1, u_k = 1 + 1/a_kk lost the low
// bits of 1/a_kk in the pivot row and column).  Row k and column k
// are published raw through parity-buffered LDS one step ahead (one barrier
// per PAIR of steps, below), and the step loop is unrolled by 8 so every
// in-tile index (k % 8) is static: publishing is a predicated store, not a
// register pick.  57 us per block (the earlier LU + two
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

// 1 / pivot: v_rcp_f64 + two Newton steps (within an ulp of the IEEE
// quotient; the refinement absorbs the rest) -- 3 dependent FMAs instead of
// the ~8-deep IEEE division sequence on the critical path of every column
__device__ __forceinline__ double gj_recip(double piv) {
  double pk = __builtin_amdgcn_rcp(piv);
  pk = fma(pk, fma(-piv, pk, 1.0), pk);
  return fma(pk, fma(-piv, pk, 1.0), pk);
}

// ---- two Gauss-Jordan steps per barrier ----------------------------------------
// The same uniform rank-1 steps, paired: rows k, k+1 and columns k, k+1 of
// the block are published raw (before step k) behind ONE barrier, and every
// thread derives step k+1's operands itself -- column k+1 and row k+1 after
// step k are one FMA each from the published values (c1_i = a_i,k+1 - g_i
// u_k+1, r1_j = a_k+1,j - g_k+1 u_j, pivot a_k+1,k+1 - g_k+1 u_k+1), exactly
// the FMAs their owners perform in the one-step form -- then applies
// a -= g u^T + g' u'^T.  Every element sees the same operation sequence as
// one Gauss-Jordan step per barrier would give it (bit-identical results),
// with half the barriers.
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
  // step k without cancellation: a' = b - G U^T with U_j = a_kj p (U_k = p),
  // G_i = a_ik (G_k = -1) and the base b = a with row k and column k zeroed
  // (the uniform form's 1 + p and a_kk - 1 lost the low bits of p: |D A - I|
  // 1.6e-10 instead of 1.8e-13 on a cond-1e4 Schur block, which cost the
  // refinement up to 6 corrections, profiles/rbt_seeds_r6.txt)
  u[KK] = kcol ? pk : u[KK];
  g[KK % TR] = krow ? -1.0 : g[KK % TR];
  // step k applied to column k+1 (rows of this tile), row k+1 (columns of
  // this tile) and the next pivot; a_k,k+1 and a_k+1,k sit in the zeroed
  // row / column, so their bases are 0
  const double uk1 = ak1 * pk;  // u[k+1]
  const double gk1 = a1k;       // g[k+1]
  g1[KK % TR] = krow ? 0.0 : g1[KK % TR];
  u1[KK] = kcol ? 0.0 : u1[KK];
#pragma unroll
  for (int i = 0; i < TR; ++i) g1[i] = fma(-g[i], uk1, g1[i]);
#pragma unroll
  for (int j = 0; j < kTl; ++j) u1[j] = fma(-gk1, u[j], u1[j]);
  const double pk1 = gj_recip(fma(-gk1, uk1, a11));
#pragma unroll
  for (int j = 0; j < kTl; ++j) u1[j] *= pk1;
  u1[KK + 1] = kcol ? pk1 : u1[KK + 1];
  g1[(KK + 1) % TR] = krow ? -1.0 : g1[(KK + 1) % TR];
  // row k+1 and column k+1 are step k+1's alone (base 0, no step-k term);
  // rows / columns k and k+1 of the tile start from 0
  g[(KK + 1) % TR] = krow ? 0.0 : g[(KK + 1) % TR];
  u[KK + 1] = kcol ? 0.0 : u[KK + 1];
  if (krow) {  // one wave in eight holds rows k, k+1: the others branch past
#pragma unroll
    for (int j = 0; j < kTl; ++j) {
      a[KK % TR][j] = 0.0;
      a[KK % TR + 1][j] = 0.0;
    }
  }
#pragma unroll
  for (int i = 0; i < TR; ++i) {
    a[i][KK] = kcol ? 0.0 : a[i][KK];
    a[i][KK + 1] = kcol ? 0.0 : a[i][KK + 1];
  }
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

// The inverse of the NB x NB block at Ablk (two Gauss-Jordan steps per
// barrier, 4 x 8 tiles on 512 threads: 57.0 us alone, profiles/gj_pair_r4.txt;
// the round-4 alternatives -- one step per barrier, 8 x 8 / 2 x 8 tiles, the
// blocked MFMA form with 16- or 32-pivot blocks -- were slower or, blocked,
// cost the refinement extra corrections, profiles/gj_blocked_r4.txt).  `col`
// (its first global column) only labels a non-finite result in info.
int block_inv(const double* Ablk, int64_t lda, int64_t col, double* Di, int* info, hipStream_t s) {
  hipLaunchKernelGGL((diag_inv_pair_kernel<4>), dim3(1), dim3(16 * NB / 4), 0, s, Ablk, lda, (int)col, Di, info);
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

// ---- split block triangular solve: the chain does only the last blocks ----------
//
// The same solve as blk_trsv_kernel, with the off-diagonal work spread over
// the chip.  In blk_trsv_kernel workgroup w reads ALL w blocks of its block row
// through one CU (8 MB for the last row at 8192): the chain step is bound by
// one CU's share of HBM bandwidth, 332 us per 8192 triangle against a ~55 us
// bandwidth floor (profiles/rbt_trace_8192_r4.txt).  Here every block row b
// has K helper workgroups: helper h accumulates F_bi x_i for the blocks i < w
// - kChainOwn with i = h (mod K), as soon as each x_i is published, and
// publishes its 128 partial sums through a sentinel-filled buffer; the chain
// workgroup applies only the last kChainOwn blocks (the ones that arrive
// last), adds the K partials in a fixed order (deterministic), multiplies by
// the stored inverse and publishes x_b.  The chain step is then a hand-off, a
// 128 x 128 mat-vec out of registers and the finish, while the F stream runs
// on up to K + 1 CUs per block row.
constexpr int kChainOwn = 2;  // blocks the chain workgroup applies itself
constexpr int kMaxHelpers = 4;

// Lanes poll their OWN published value p[lane] until it is not the
// sentinel (bounded like settle_x); false when the spin ran out or another
// workgroup reported an error.
__device__ __forceinline__ bool settle_own(const double* __restrict__ p, int* err, double& out) {
  const unsigned long long* pp = reinterpret_cast<const unsigned long long*>(p);
  unsigned long long v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool ok = true;
  if (__ballot(v == kSentinel) != 0) {
    const unsigned long long t0 = rtc();
    while (__ballot(v == kSentinel) != 0) {
      __builtin_amdgcn_s_sleep(1);
      if (v == kSentinel) v = __hip_atomic_load(pp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (rtc() - t0 > kSpinTicks || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        if (__lane_id() == 0) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = false;
        break;
      }
    }
  }
  out = __builtin_bit_cast(double, v);
  return ok;
}

// grid = nblk * (K + 1): ids [0, nblk) are the chain (position w = id), ids
// nblk + K w + h the helpers of position w.  hpart: nblk * K * 128 doubles,
// sentinel-filled.  Requires the whole grid co-resident (checked by the host).
template <typename T, bool UPPER>
__global__ __launch_bounds__(kDT) void blk_trsv_split_kernel(const T* __restrict__ F, int64_t ldf,
                                                            const double* __restrict__ Dinv,
                                                            const double* __restrict__ c, double* __restrict__ x,
                                                            double* __restrict__ ysave, double* __restrict__ hpart,
                                                            int nblk, int K, int* __restrict__ err,
                                                            const double* __restrict__ G,
                                                            const double* __restrict__ zlast) {
  __shared__ double part[4][NB];
  __shared__ double rb[NB];
  __shared__ int bad;
  const int t = threadIdx.x, r = t & (NB - 1), lane = t & 63;
  const int q = __builtin_amdgcn_readfirstlane(t >> 7);
  const int id = blockIdx.x;
  const bool chain = id < nblk;
  const int w = chain ? id : (id - nblk) / K;
  const int h = chain ? 0 : (id - nblk) % K;
  if (w >= nblk) return;
  const int b = UPPER ? nblk - 1 - w : w;
  const int row = NB * b + r;
  if (t == 0) bad = 0;
  const int own0 = w > kChainOwn ? w - kChainOwn : 0;  // the chain applies blocks own0 .. w-1
  const T* frow = F + (int64_t)row * ldf + kQW * q;
  auto blk = [&](int i) { return frow + (int64_t)NB * (UPPER ? nblk - 1 - i : i); };
  auto xidx = [&](int i) { return NB * (UPPER ? nblk - 1 - i : i) + kQW * q; };
  double acc = 0.0;
  bool ok = true;
  T ua[kQW], ub[kQW];
  auto step = [&](const T(&u)[kQW], unsigned long long v, int i, bool nap) -> bool {
    double xl;
    if (!settle_x(x, xidx(i), v, err, xl, nap)) return false;
#pragma unroll
    for (int j = 0; j < kQW; ++j) acc = fma(-(double)u[j], bcast_lane(xl, j), acc);
    return true;
  };

  if (!chain) {
    // helper h of position w: blocks i = h, h + K, ... < own0, next block's
    // factor loads in flight under the current one's wait
    int i = h;
    if (i < own0) load_blk(ua, blk(i));
    for (; i + K < own0; i += 2 * K) {
      unsigned long long v = issue_x(x, xidx(i));
      load_blk(ub, blk(i + K));
      if (!step(ua, v, i, true)) { ok = false; break; }
      v = issue_x(x, xidx(i + K));
      if (i + 2 * K < own0) load_blk(ua, blk(i + 2 * K));
      if (!step(ub, v, i + K, true)) { ok = false; break; }
    }
    if (ok && i < own0) ok = step(ua, issue_x(x, xidx(i)), i, true);
    part[q][r] = acc;
    if (!ok && lane == 0) bad = 1;
    __syncthreads();
    if (bad) return;
    if (q == 0) {
      double s = part[0][r] + part[1][r] + part[2][r] + part[3][r];
      if (__builtin_bit_cast(unsigned long long, s) == kSentinel) s = __builtin_nan("");
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(hpart + ((int64_t)w * K + h) * NB + r),
                         __builtin_bit_cast(unsigned long long, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  // chain: this block's inverse rows and right-hand side first, pinned
  double dv[kQW];
  {
    const double* d = Dinv + ((int64_t)b * NB + r) * NB + kQW * q;
#pragma unroll
    for (int j = 0; j < kQW; ++j) dv[j] = d[j];
  }
  double cv = c[row];
  if (zlast != nullptr && b > 0) {
    // the forward solve (G form) left y_b without its last block's product:
    // c_b -= F_{b,b-1} z_{b-1}, formed here while this row waits its turn
    load_blk(ua, F + (int64_t)row * ldf + (int64_t)(b - 1) * NB + kQW * q);
    const double* zp = zlast + (int64_t)(b - 1) * NB + kQW * q;
    double f0 = 0.0, f1 = 0.0;
#pragma unroll
    for (int j = 0; j < kQW; j += 2) {
      f0 = fma((double)ua[j], zp[j], f0);
      f1 = fma((double)ua[j + 1], zp[j + 1], f1);
    }
    part[q][r] = f0 + f1;
    __syncthreads();
    cv -= part[0][r] + part[1][r] + part[2][r] + part[3][r];
    __syncthreads();  // part is reused below
  }
#pragma unroll
  for (int j = 0; j < kQW; ++j) asm volatile("" : "+v"(dv[j]));
  asm volatile("" : "+v"(cv));
  // the helpers' partials are read early -- after block w-2, while x_{w-1} is
  // still on its way -- so a ready partial costs no load on the chain
  unsigned long long hb[kMaxHelpers];
  auto prefetch_h = [&]() {
    if (q == 0) {
#pragma unroll
      for (int hh = 0; hh < kMaxHelpers; ++hh)
        hb[hh] = hh < K ? __hip_atomic_load(reinterpret_cast<const unsigned long long*>(
                                                hpart + ((int64_t)w * K + hh) * NB + r),
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0ull;
    }
  };
  if (G != nullptr && w > 0) {
    // x_b = v - G x_{w-1}: v = Dinv_b (c_b - sum_{i < w-1} F_bi x_i) is formed
    // while x_{w-1} is on its way, and the step after the last hand-off is one
    // 128 x 128 mat-vec with G = Dinv_b F_{b,w-1} (gprod_kernel) and one
    // barrier, instead of two mat-vecs and four barriers
    double gv[kQW];
    {
      const double* gp = G + (((int64_t)(UPPER ? 1 : 0) * nblk + b) * NB + r) * NB + kQW * q;
#pragma unroll
      for (int j = 0; j < kQW; ++j) gv[j] = gp[j];
    }
    if (w >= 2) {
      load_blk(ua, blk(w - 2));
      ok = step(ua, issue_x(x, xidx(w - 2)), w - 2, true);
    }
    prefetch_h();
    part[q][r] = acc;
    if (!ok && lane == 0) bad = 1;
    __syncthreads();
    if (bad) return;
    double y0 = 0.0;
    if (q == 0) {
      y0 = cv + part[0][r] + part[1][r] + part[2][r] + part[3][r];
#pragma unroll
      for (int hh = 0; hh < kMaxHelpers; ++hh) {
        if (hh >= K || !ok) break;
        double hpv = __builtin_bit_cast(double, hb[hh]);
        if (__ballot(hb[hh] == kSentinel) != 0) ok = settle_own(hpart + ((int64_t)w * K + hh) * NB + r, err, hpv);
        y0 += hpv;
      }
      if (!ok && lane == 0) bad = 1;
      rb[r] = y0;
      // the forward solve keeps y_b less its last product (the backward
      // solve's chain adds F_{b,b-1} z_{b-1} itself: zlast)
      if (ysave) ysave[row] = y0;
    }
    __syncthreads();
    if (bad) return;
    double xs = 0.0;
#pragma unroll
    for (int j = 0; j < kQW; ++j) xs = fma(dv[j], rb[kQW * q + j], xs);
    __syncthreads();
    part[q][r] = xs;
    __syncthreads();
    const double v = q == 0 ? part[0][r] + part[1][r] + part[2][r] + part[3][r] : 0.0;
    __syncthreads();  // part is rewritten below
    double xl;
    ok = settle_x(x, xidx(w - 1), issue_x(x, xidx(w - 1)), err, xl, false);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < kQW; j += 2) {
      s0 = fma(gv[j], bcast_lane(xl, j), s0);
      s1 = fma(gv[j + 1], bcast_lane(xl, j + 1), s1);
    }
    part[q][r] = s0 + s1;
    if (!ok && lane == 0) bad = 1;
    __syncthreads();
    if (bad) return;
    if (q == 0) {
      double xv = v - (part[0][r] + part[1][r] + part[2][r] + part[3][r]);
      if (__builtin_bit_cast(unsigned long long, xv) == kSentinel) xv = __builtin_nan("");
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + row), __builtin_bit_cast(unsigned long long, xv),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  // the last kChainOwn (= 2) blocks, in chain order
  if (own0 + 1 < w) {
    load_blk(ua, blk(own0));
    unsigned long long v = issue_x(x, xidx(own0));
    load_blk(ub, blk(own0 + 1));
    ok = step(ua, v, own0, true);
    prefetch_h();
    if (ok) ok = step(ub, issue_x(x, xidx(own0 + 1)), own0 + 1, false);
  } else {
    prefetch_h();
    if (own0 < w) {
      load_blk(ua, blk(own0));
      ok = step(ua, issue_x(x, xidx(own0)), own0, false);
    }
  }
  part[q][r] = acc;
  if (!ok && lane == 0) bad = 1;
  __syncthreads();
  if (bad) return;
  if (q == 0) {
    // the helpers' partials, added in helper order after the chain's own
    // blocks: the same sum in every run
    double y = cv + part[0][r] + part[1][r] + part[2][r] + part[3][r];
#pragma unroll
    for (int hh = 0; hh < kMaxHelpers; ++hh) {
      if (hh >= K || !ok) break;
      double hp = __builtin_bit_cast(double, hb[hh]);
      if (__ballot(hb[hh] == kSentinel) != 0) ok = settle_own(hpart + ((int64_t)w * K + hh) * NB + r, err, hp);
      y += hp;
    }
    if (!ok && lane == 0) bad = 1;
    rb[r] = y;
    if (ysave) ysave[row] = y;
  }
  __syncthreads();
  if (bad) return;
  double xs = 0.0;
#pragma unroll
  for (int j = 0; j < kQW; ++j) xs = fma(dv[j], rb[kQW * q + j], xs);
  __syncthreads();
  part[q][r] = xs;
  __syncthreads();
  if (q == 0) {
    double xv = part[0][r] + part[1][r] + part[2][r] + part[3][r];
    if (__builtin_bit_cast(unsigned long long, xv) == kSentinel) xv = __builtin_nan("");
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + row), __builtin_bit_cast(unsigned long long, xv),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// G[d][b] = Dinv_b F_{b,b-1} (d = 0, the forward solve's last block) and
// Dinv_b F_{b,b+1} (d = 1, the backward solve's), row-major 128 x 128, on
// the fp64 matrix cores: 4 waves of 64 x 64 (4 x 4 v_mfma_f64_16x16x4f64
// blocks), operands straight from L2 (one launch per factorisation).
__global__ __launch_bounds__(256) void gprod_kernel(const double* __restrict__ F, int64_t ldf,
                                                    const double* __restrict__ Dinv, double* __restrict__ G,
                                                    int nblk) {
  const int b = blockIdx.x, d = blockIdx.y;
  const int nb = d == 0 ? b - 1 : b + 1;
  if (nb < 0 || nb >= nblk) return;
  const double* A = Dinv + (int64_t)b * NB * NB;
  const double* B = F + (int64_t)b * NB * ldf + (int64_t)nb * NB;
  double* C = G + ((int64_t)d * nblk + b) * NB * NB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64, r16 = lane & 15, q = lane >> 4;
  dev::d4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = dev::d4{0.0, 0.0, 0.0, 0.0};
  for (int k0 = 0; k0 < NB; k0 += 4) {
    double af[4], bf[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = A[(wm + 16 * i + r16) * NB + k0 + q];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = B[(int64_t)(k0 + q) * ldf + wn + 16 * j + r16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(wm + 16 * i + q + 4 * r) * NB + wn + 16 * j + r16] = acc[i][j][r];
}

__global__ __launch_bounds__(256) void fill_sentinel2_kernel(unsigned long long* __restrict__ a, int na,
                                                             unsigned long long* __restrict__ b, int nb) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < na) a[i] = kSentinel;
  if (i < nb) b[i] = kSentinel;
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

// Block LDU factorisation of the transformed (fp64) matrix in place, no
// lookahead (below 32 blocks): per block k, Dinv_k = A_kk^-1 (Gauss-Jordan),
// W = A_kk^-1 A_k,rest and A_rest,rest -= A_rest,k W on the fp64 matrix cores
// (dgemm.hip v_mfma_f64_16x16x4f64).
int factor_impl(double* M, int64_t ldm, int64_t np, double* Dinv, double* W, int* info, hipStream_t s) {
  for (int64_t k0 = 0; k0 < np; k0 += NB) {
    double* Di = Dinv + (k0 / NB) * NB * NB;
    GELIM_TRY(diag_inv(M, ldm, k0, Di, info, s));
    const int64_t rest = np - k0 - NB;
    if (rest <= 0) break;
    double* A12 = M + k0 * ldm + k0 + NB;
    double* A21 = M + (k0 + NB) * ldm + k0;
    double* A22 = M + (k0 + NB) * ldm + k0 + NB;
    GELIM_TRY(dgemm_ex(W, rest, Di, NB, A12, ldm, NB, rest, NB, 1.0, 0, s));        // W = A11^-1 A12
    GELIM_TRY(dgemm_ex(A22, ldm, A21, ldm, W, rest, rest, rest, NB, -1.0, 1, s));  // A22 -= A21 W
  }
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
               hipStream_t side, hipEvent_t e0, hipEvent_t e1) {
  const int64_t nblk = np / NB;
  GELIM_TRY(diag_inv(M, ldm, 0, Dinv, info, s));
  bool side_used = false;
  for (int64_t k = 0, pair = 0; k + 1 < nblk; k += 2, ++pair) {
    const int64_t k0 = k * NB, r1 = np - k0 - NB;  // columns right of block k
    double* Wp = W4 + (pair & 1) * 2 * NB * np;    // 2 NB rows, ld r1
    double* Ak = M + (k0 + NB) * ldm + k0;         // A[k+1:, k]
    GELIM_TRY(dgemm_ex(Wp, r1, Dinv + k * NB * NB, NB, M + k0 * ldm + k0 + NB, ldm, NB, r1, NB, 1.0, 0, s));
    // step k on block k+1: its column (rows k+1..), its row (columns k+2..),
    // one launch (disjoint outputs, shared operands)
    const int64_t r2 = r1 - NB;  // columns right of block k+1
    GELIM_TRY(dgemm_pair(GemmOp{M + (k0 + NB) * ldm + k0 + NB, ldm, Ak, ldm, Wp, r1, r1, NB, NB},
                         GemmOp{M + (k0 + NB) * ldm + k0 + 2 * NB, ldm, Ak, ldm, Wp + NB, r1, r2 > 0 ? NB : 0, r2, NB},
                         -1.0, 1, s));
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
    // the panel's block columns and block rows: one launch
    GELIM_TRY(dgemm_pair(GemmOp{M + (k0 + 2 * NB) * ldm + k0 + 2 * NB, ldm, A2, ldm, Wp + NB, r1, r2, pw, 2 * NB},
                         GemmOp{M + (k0 + 2 * NB) * ldm + k0 + 2 * NB + pw, ldm, A2, ldm, Wp + NB + pw, r1,
                                r4 > 0 ? pw : 0, r4, 2 * NB},
                         -1.0, 1, s));
    if (r4 > 0) {
      HIP_TRY(hipEventRecord(e0, s));
      HIP_TRY(hipStreamWaitEvent(side, e0, 0));
      GELIM_TRY(dgemm_ex(M + (k0 + 2 * NB + pw) * ldm + k0 + 2 * NB + pw, ldm, M + (k0 + 2 * NB + pw) * ldm + k0, ldm,
                         Wp + NB + pw, r1, r4, r4, 2 * NB, -1.0, 1, side));
      HIP_TRY(hipEventRecord(e1, side));
      side_used = true;
    }
    GELIM_TRY(diag_inv(M, ldm, k0 + 2 * NB, Dinv + (k + 2) * NB * NB, info, s));
  }
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
               double* x, unsigned* flags, hipStream_t s, double* hp = nullptr, const double* G = nullptr) {
  const int nblk = (int)(np / NB);
  // the split form (blk_trsv_split_kernel) when its grid of nblk (K + 1)
  // workgroups fits at once, with as many helpers per block row as fit
  static const int split_per_cu = [] {
    int a = 0, b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, blk_trsv_split_kernel<T, false>, kDT, 0) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, blk_trsv_split_kernel<T, true>, kDT, 0) != hipSuccess)
      return 0;
    return std::min(a, b);
  }();
  int K = 0;
  if (hp && split_per_cu > 0 && nblk <= kMaxBlocks)
    for (int k = kMaxHelpers; k >= 1 && K == 0; --k)
      if (coresident(split_per_cu, (int64_t)nblk * (k + 1))) K = k;
  if (K > 0) {
    int* err = reinterpret_cast<int*>(flags);
    const int nh = nblk * K * NB;  // helper partials per direction
    const bool alias = x == c;
    const unsigned g = (unsigned)((std::max<int64_t>(np, 2 * (int64_t)nh) + 255) / 256);
    hipLaunchKernelGGL(fill_sentinel2_kernel, dim3(g), dim3(256), 0, s, reinterpret_cast<unsigned long long*>(z),
                       (int)np, reinterpret_cast<unsigned long long*>(hp), 2 * nh);
    if (!alias)
      hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s,
                         reinterpret_cast<unsigned long long*>(x), (int)np);
    HIP_TRY(hipGetLastError());
    const unsigned grid = (unsigned)(nblk * (K + 1));
    hipLaunchKernelGGL((blk_trsv_split_kernel<T, false>), dim3(grid), dim3(kDT), 0, s, M, ldm, Dinv, c, z, y, hp,
                       nblk, K, err, G, (const double*)nullptr);
    HIP_TRY(hipGetLastError());
    if (alias) {
      hipLaunchKernelGGL(fill_sentinel_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s,
                         reinterpret_cast<unsigned long long*>(x), (int)np);
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL((blk_trsv_split_kernel<T, true>), dim3(grid), dim3(kDT), 0, s, M, ldm, Dinv, y, x,
                       (double*)nullptr, hp + nh, nblk, K, err, G, G ? (const double*)z : nullptr);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  static const bool fits = [] {
    int a = 0, b = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, blk_trsv_kernel<T, false>, kDT, 0) == hipSuccess &&
           hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, blk_trsv_kernel<T, true>, kDT, 0) == hipSuccess &&
           a >= 1 && b >= 1;
  }();
  // the XCD-packed chain maps positions across the whole 8 x 32 grid (position
  // 32 is workgroup 1, waiting on position 31 = workgroup 248), so it needs
  // every one of them resident; one workgroup per block row needs only nblk
  // (workgroups are dispatched in order, each waits on lower ids only)
  if (!fits || nblk > kMaxBlocks) return kNotResident;
  const int pack = coresident(1, 8 * kXcdSlots) ? 1 : 0;
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
  double* M = nullptr;      // np x ldm: the transformed matrix, then its block-LDU factor
  double* Dinv = nullptr;   // nblk x NB x NB: inverse of every (Schur) diagonal block
  double* W = nullptr;      // 4 x NB x np: A_kk^-1 A_k,rest (pairs of blocks, double-buffered under lookahead)
  double* ud = nullptr;     // U's butterfly diagonals (8 x np/4)
  double* vd = nullptr;     // V's
  unsigned* flags = nullptr;  // [0]: the solves' error word
  double* hp = nullptr;       // split solves' helper partials (2 x kMaxBlocks x kMaxHelpers x NB)
  double* G = nullptr;        // 2 x nblk x NB x NB: Dinv_b F_{b,b-1}, Dinv_b F_{b,b+1} (gprod_kernel)
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
  int lookahead = 0;        // lookahead over pairs of blocks on a side stream (factor_la2)
  hipStream_t side = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
};

extern "C" int64_t gelim_mixed_max_n(void) { return (int64_t)gelim::kMaxBlocks * gelim::NB; }

extern "C" void gelim_mixed_plan_destroy(gelim_mixed_plan* p) {
  if (!p) return;
  for (void* q : {(void*)p->M, (void*)p->Dinv, (void*)p->W, (void*)p->ud, (void*)p->vd,
                  (void*)p->rv, (void*)p->wv, (void*)p->dv, (void*)p->xb, (void*)p->om, (void*)p->flags, (void*)p->c,
                  (void*)p->y, (void*)p->z, (void*)p->xs, (void*)p->info, (void*)p->hp, (void*)p->G})
    (void)hipFree(q);
  if (p->e0) (void)hipEventDestroy(p->e0);
  if (p->e1) (void)hipEventDestroy(p->e1);
  if (p->side) (void)hipStreamDestroy(p->side);
  delete p;
}

// n: order of the system; ud / vd: host arrays of 8 * np/4 butterfly entries
// each (np = gelim_mixed_padded(n)), exp(r/10) with r uniform in [-1/2, 1/2].
extern "C" int64_t gelim_mixed_padded(int64_t n) { return (n + gelim::kPadTo - 1) / gelim::kPadTo * gelim::kPadTo; }

// fp64 must be 1 (fp64 factors; the fp32-factor engine was removed).
extern "C" gelim_mixed_plan* gelim_mixed_plan_create2(int64_t n, const double* ud, const double* vd, int fp64) {
  const int64_t np = gelim_mixed_padded(n);
  if (n <= 0 || np > gelim_mixed_max_n()) {
    GELIM_FAIL(GELIM_E_ARG, "mixed plan: n must be in [1, " + std::to_string(gelim_mixed_max_n()) +
                                "] (persistent triangular solves: every 128-row block resident)");
    return nullptr;
  }
  if (!fp64) {
    GELIM_FAIL(GELIM_E_ARG, "mixed plan: fp32 factors (the former hip-mixed engine) were removed in round 5 -- "
                            "slower than fp64 hip-rbt at every n and not convergent at 16384; use fp64 = 1");
    return nullptr;
  }
  auto* p = new gelim_mixed_plan;
  p->n = n;
  p->np = np;
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
  // lookahead from 24 blocks (n = 3072; round 5, with the grouped critical
  // GEMMs: 3072 2.72 vs 2.83 ms, 2048 1.70 vs 1.65, trsv_split_r5.txt): below
  // it the side stream's share is too small to pay for the cross-stream waits.  The side GEMMs run on an uncapped grid
  // (8192 15.0 ms vs 18.7 with 64 CUs reserved for the chain); CU masks,
  // stream priorities, a third stream for the updates the next inverse does
  // not read, and one-block (instead of pair) lookahead were all measured
  // slower in rounds 3-4 (profiles/rbt_engine_round3.txt, stream_prio_r4.txt).
  p->lookahead = np >= 3072;
  if (p->lookahead) {
    if (gelim::side_stream_create(&p->side) != GELIM_OK) return fail("side stream");
    if (hipEventCreateWithFlags(&p->e0, hipEventDisableTiming) != hipSuccess) return fail("event");
    if (hipEventCreateWithFlags(&p->e1, hipEventDisableTiming) != hipSuccess) return fail("event");
  }
  if (hipMalloc((void**)&p->ud, sizeof(double) * nd) != hipSuccess) return fail("ud");
  if (hipMalloc((void**)&p->vd, sizeof(double) * nd) != hipSuccess) return fail("vd");
  (void)nblk;
  if (hipMalloc((void**)&p->flags, 16) != hipSuccess) return fail("flags");
  if (hipMalloc((void**)&p->c, sizeof(double) * np) != hipSuccess) return fail("c");
  if (hipMalloc((void**)&p->y, sizeof(double) * np) != hipSuccess) return fail("y");
  if (hipMalloc((void**)&p->z, sizeof(double) * np) != hipSuccess) return fail("z");
  if (hipMalloc((void**)&p->xs, sizeof(double) * np) != hipSuccess) return fail("xs");
  if (hipMalloc((void**)&p->hp, sizeof(double) * 2 * gelim::kMaxBlocks * gelim::kMaxHelpers * gelim::NB) !=
      hipSuccess)
    return fail("helper partials");
  if (hipMalloc((void**)&p->G, 2 * sizeof(double) * (size_t)np * gelim::NB) != hipSuccess) return fail("G blocks");
  if (hipMalloc((void**)&p->info, 16) != hipSuccess) return fail("info");
  for (double** b : {&p->rv, &p->wv, &p->dv, &p->xb})
    if (hipMalloc((void**)b, sizeof(double) * (size_t)n) != hipSuccess) return fail("refinement vectors");
  if (hipMalloc((void**)&p->om, 16) != hipSuccess) return fail("omega");
  if (hipMemcpy(p->ud, ud, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("ud copy");
  if (hipMemcpy(p->vd, vd, sizeof(double) * nd, hipMemcpyHostToDevice) != hipSuccess) return fail("vd copy");
  return p;
}

extern "C" gelim_mixed_plan* gelim_mixed_plan_create(int64_t n, const double* ud, const double* vd) {
  return gelim_mixed_plan_create2(n, ud, vd, 1);
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
  const dim3 grid((unsigned)((h + 255) / 256), (unsigned)h);
  hipLaunchKernelGGL(rbt_matrix_kernel<double>, grid, dim3(256), 0, s, aug, ld, (int)p->n, (int)np, p->ud, p->vd,
                     p->M, ldm);
  HIP_TRY(hipGetLastError());
  if (p->lookahead)
    GELIM_TRY(factor_la2(p->M, ldm, np, p->Dinv, p->W, p->info, s, p->side, p->e0, p->e1));
  else
    GELIM_TRY(factor_impl(p->M, ldm, np, p->Dinv, p->W, p->info, s));
  // the solves' last-block products (split solves only read them)
  if (np > NB) {
    hipLaunchKernelGGL(gprod_kernel, dim3((unsigned)(np / NB), 2), dim3(256), 0, s, p->M, ldm, p->Dinv, p->G,
                       (int)(np / NB));
    HIP_TRY(hipGetLastError());
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
  const int rc = solve_impl<double>(p->M, p->ldm, np, p->Dinv, p->c, p->z, p->y, p->xs, p->flags, s, p->hp,
                                    np > NB ? p->G : nullptr);
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
