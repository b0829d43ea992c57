// fp64 GEMM for THIN problems on the CDNA4 matrix cores: C (+)= alpha A B
// when one of M, N is ~128 and K <= 256 -- the block-column / block-row
// updates and W = D^-1 A12 products of the randomised block-LDU engine
// (lu_mixed.hip factor_la2: 8192 x 128 x 128, 128 x 8064 x 128, 7936 x 256 x
// 256 ...) and of its distributed form (parallel/dist_rbt.py).  Those shapes
// give dgemm.hip's LDS-tiled kernel fewer tiles than CUs, and its K loop (one
// barrier and one exposed global-load round trip per 16-deep K step) then
// dominates: ~7 TFLOP/s (profiles/rbt_trace_8192.txt, 194 calls = 7.5 ms of
// the 12.6 ms main queue at 8192).
//
// This kernel has no LDS and no barrier: every wave owns a (16 MB) x (16 NB)
// tile of C and feeds v_mfma_f64_16x16x4f64 straight from registers.  The
// f64 MFMA operand maps (cdna_hip_programming.md §3) put A[l & 15][k = l >> 4]
// and B[k = l >> 4][l & 15] in lane l; the reduction order over k is free, so
// lane group q = l >> 4 takes a CONTIGUOUS run of KC k's per chunk (k = 4 KC c
// + KC q + s): its A operands are one 16-byte-vectorised row segment, its B
// operands 16 consecutive columns (one 128-byte line per k across the 16
// lanes).  Chunks are double-buffered in registers, so one load round trip
// is exposed per kernel instead of one per K step, and small tiles give 4-16x
// the waves of the 64 x 64 LDS tiles.  C is read before the K loop (one
// round trip under the A / B loads) and written once.
//
// Reference loop this replaces: the rank-1 update `matrix[j][k] -= pivotval *
// matrix[i][k]` (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:172-180),
// here as rank-128 / rank-256 block products.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

struct ThinArgs {
  double* C;
  int64_t ldc;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  int M, N, K;
  int tiles_n, ntiles;
  double alpha;
  int acc;
};

template <int MB, int NB, int KC>
struct Chunk {
  double a[MB][KC];
  double b[NB][KC];
};

template <int MB, int NB, int KC>
__device__ __forceinline__ void load_chunk(Chunk<MB, NB, KC>& ch, const double* const (&arow)[MB],
                                           const double* const (&bcol)[NB], int64_t ldb, int k0) {
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int s = 0; s < KC; s += 2) {
      const double2 v = *reinterpret_cast<const double2*>(arow[i] + k0 + s);
      ch.a[i][s] = v.x;
      ch.a[i][s + 1] = v.y;
    }
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int s = 0; s < KC; ++s) ch.b[j][s] = bcol[j][(int64_t)(k0 + s) * ldb];
}

template <int MB, int NB, int KC>
__device__ __forceinline__ void mma_chunk(dev::d4 (&acc)[MB][NB], const Chunk<MB, NB, KC>& ch) {
#pragma unroll
  for (int s = 0; s < KC; ++s)
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(ch.a[i][s], ch.b[j][s], acc[i][j], 0, 0, 0);
}

template <int MB, int NB, int KC>
__global__ __launch_bounds__(256) void dgemm_thin_kernel(ThinArgs g) {
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= g.ntiles) return;
  const int tr = wid / g.tiles_n, tc = wid - tr * g.tiles_n;
  const int m0 = tr * 16 * MB, n0 = tc * 16 * NB;
  const int r = lane & 15, q = lane >> 4;
  // operand rows / columns (clamped at the edges: their products are never stored)
  const double* arow[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) arow[i] = g.A + (int64_t)min(m0 + 16 * i + r, g.M - 1) * g.lda + KC * q;
  const double* bcol[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) bcol[j] = g.B + (int64_t)(KC * q) * g.ldb + min(n0 + 16 * j + r, g.N - 1);
  const int nch = g.K / (4 * KC);
  Chunk<MB, NB, KC> c0, c1;
  load_chunk<MB, NB, KC>(c0, arow, bcol, g.ldb, 0);
  // C behind the first chunk's loads (vmcnt is in order)
  dev::d4 cv[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = min(n0 + 16 * j + r, g.N - 1);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = min(m0 + 16 * i + q + 4 * rr, g.M - 1);
        cv[i][j][rr] = g.acc ? g.C[(int64_t)row * g.ldc + col] : 0.0;
      }
    }
  dev::d4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = dev::d4{0.0, 0.0, 0.0, 0.0};
  // chunk loop unrolled by two: the register double buffer keeps static indices
  for (int c = 0; c < nch; c += 2) {
    if (c + 1 < nch) load_chunk<MB, NB, KC>(c1, arow, bcol, g.ldb, (c + 1) * 4 * KC);
    mma_chunk<MB, NB, KC>(acc, c0);
    if (c + 1 >= nch) break;
    if (c + 2 < nch) load_chunk<MB, NB, KC>(c0, arow, bcol, g.ldb, (c + 2) * 4 * KC);
    mma_chunk<MB, NB, KC>(acc, c1);
  }
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + 16 * j + r;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = m0 + 16 * i + q + 4 * rr;
        if (row < g.M && col < g.N) g.C[(int64_t)row * g.ldc + col] = fma(g.alpha, acc[i][j][rr], cv[i][j][rr]);
      }
    }
}

// Deep-prefetch form: DEPTH chunks in flight (a register ring, the chunk loop
// fully unrolled up to K = 256 so every ring index is static): the K loop
// pays ceil(nch / DEPTH) memory round trips instead of nch.
template <int MB, int NB, int KC, int DEPTH>
__global__ __launch_bounds__(256) void dgemm_thin_deep_kernel(ThinArgs g) {
  constexpr int kMaxCh = 256 / (4 * KC);
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wid >= g.ntiles) return;
  const int tr = wid / g.tiles_n, tc = wid - tr * g.tiles_n;
  const int m0 = tr * 16 * MB, n0 = tc * 16 * NB;
  const int r = lane & 15, q = lane >> 4;
  const double* arow[MB];
#pragma unroll
  for (int i = 0; i < MB; ++i) arow[i] = g.A + (int64_t)min(m0 + 16 * i + r, g.M - 1) * g.lda + KC * q;
  const double* bcol[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) bcol[j] = g.B + (int64_t)(KC * q) * g.ldb + min(n0 + 16 * j + r, g.N - 1);
  const int nch = g.K / (4 * KC);
  Chunk<MB, NB, KC> ring[DEPTH];
#pragma unroll
  for (int c = 0; c < DEPTH; ++c)
    if (c < nch) load_chunk<MB, NB, KC>(ring[c], arow, bcol, g.ldb, c * 4 * KC);
  dev::d4 cv[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = min(n0 + 16 * j + r, g.N - 1);
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = min(m0 + 16 * i + q + 4 * rr, g.M - 1);
        cv[i][j][rr] = g.acc ? g.C[(int64_t)row * g.ldc + col] : 0.0;
      }
    }
  dev::d4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = dev::d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < kMaxCh; ++c) {
    if (c < nch) {
      mma_chunk<MB, NB, KC>(acc, ring[c % DEPTH]);
      if (c + DEPTH < nch) load_chunk<MB, NB, KC>(ring[c % DEPTH], arow, bcol, g.ldb, (c + DEPTH) * 4 * KC);
    }
  }
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + 16 * j + r;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int row = m0 + 16 * i + q + 4 * rr;
        if (row < g.M && col < g.N) g.C[(int64_t)row * g.ldc + col] = fma(g.alpha, acc[i][j][rr], cv[i][j][rr]);
      }
    }
}

template <int MB, int NB, int KC, int DEPTH>
int launch_deep(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                int64_t N, int64_t K, double alpha, int accumulate, hipStream_t s) {
  if (K > 256) return 1;
  const int tm = (int)((M + 16 * MB - 1) / (16 * MB)), tn = (int)((N + 16 * NB - 1) / (16 * NB));
  ThinArgs g{C, ldc, A, lda, B, ldb, (int)M, (int)N, (int)K, tn, tm * tn, alpha, accumulate ? 1 : 0};
  hipLaunchKernelGGL((dgemm_thin_deep_kernel<MB, NB, KC, DEPTH>), dim3((unsigned)((g.ntiles + 3) / 4)), dim3(256), 0,
                     s, g);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

template <int MB, int NB, int KC>
int launch_thin(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                int64_t N, int64_t K, double alpha, int accumulate, hipStream_t s) {
  const int tm = (int)((M + 16 * MB - 1) / (16 * MB)), tn = (int)((N + 16 * NB - 1) / (16 * NB));
  ThinArgs g{C, ldc, A, lda, B, ldb, (int)M, (int)N, (int)K, tn, tm * tn, alpha, accumulate ? 1 : 0};
  hipLaunchKernelGGL((dgemm_thin_kernel<MB, NB, KC>), dim3((unsigned)((g.ntiles + 3) / 4)), dim3(256), 0, s, g);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// Shapes: variant 0 picks by shape (the wave tile along the long side),
// 1..5 force (MB, NB, KC) = (2,2,4), (2,2,8), (1,4,4), (4,1,4), (2,4,4);
// 6..8 the deep-prefetch form (MB, NB, KC, DEPTH) = (1,1,4,8), (2,2,4,4), (1,2,4,6).
// Contract: K a multiple of 32 (16 for KC = 4 variants), A 16-byte aligned,
// lda even.  Returns 1 (nothing launched) when the contract does not hold.
int dgemm_thin(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
               int64_t N, int64_t K, double alpha, int accumulate, int variant, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return GELIM_OK;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return 1;
  if ((lda & 1) || (((uintptr_t)A) & 15)) return 1;
  if (variant == 0) variant = (K % 32 == 0) ? 2 : 1;
  switch (variant) {
    case 1:
      if (K % 16) return 1;
      return launch_thin<2, 2, 4>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 2:
      if (K % 32) return 1;
      return launch_thin<2, 2, 8>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 3:
      if (K % 16) return 1;
      return launch_thin<1, 4, 4>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 4:
      if (K % 16) return 1;
      return launch_thin<4, 1, 4>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 5:
      if (K % 16) return 1;
      return launch_thin<2, 4, 4>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 6:  // deep prefetch: every K chunk of a 16 x 16 wave tile in flight (K <= 128)
      if (K % 16) return 1;
      return launch_deep<1, 1, 4, 8>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 7:
      if (K % 16) return 1;
      return launch_deep<2, 2, 4, 4>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    case 8:
      if (K % 16) return 1;
      return launch_deep<1, 2, 4, 6>(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, s);
    default:
      return 1;
  }
}

}  // namespace gelim

// Tests / microbenchmarks: the thin kernel with an explicit variant (0 =
// automatic); returns 1 when the shape / alignment is outside its contract.
extern "C" int gelim_gpu_dgemm_thin(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb,
                                    int64_t M, int64_t N, int64_t K, double alpha, int accumulate, int variant,
                                    void* stream) {
  return gelim::dgemm_thin(C, ldc, A, lda, B, ldb, M, N, K, alpha, accumulate, variant, (hipStream_t)stream);
}
