// fp64 GEMM on the CDNA4 matrix cores: C += alpha * A * B (alpha = +-1),
// row-major operands with arbitrary leading dimensions.  This is the trailing
// update A22 -= L21 * U12 of the wide-panel blocked LU (biglu.hip) -- the
// reference's O(n^3) hot loop `matrix[j][k] -= pivotval * matrix[i][k]`
// (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:172-180) with nb
// rank-1 updates fused into one rank-nb product -- and of the distributed
// solver's per-block update.
//
// Shape of the kernel (measured, tools/microbench/mfma_f64.hip): one wave
// issues a v_mfma_f64_16x16x4_f64 every 64 cycles whatever the number of
// independent accumulators, two waves on a SIMD interleave to one per 32
// cycles (77 TFLOP/s chip-wide).  So the kernel runs two 256-thread
// workgroups per CU (2 waves per SIMD, <= 256 VGPRs per lane):
//  * workgroup tile 128 x 128, 4 waves as 2 x 2, each wave 64 x 64 = 4 x 4
//    blocks of the 16x16x4 f64 MFMA (64 accumulator doubles per lane);
//  * K in steps of BK = 16, A and B tiles double-buffered in LDS (one barrier
//    per step); A is stored transposed ([k][m]) and negated when alpha < 0,
//    B as is ([k][n]); rows padded to 144 doubles so the two 16-lane halves
//    of every ds_read_b64 land on disjoint bank sets; the transposed A tile
//    is XOR-swizzled (column m ^ (k & 14)) so its ds_write_b64 stores are
//    conflict-free (unswizzled: 8-way, 64 % of the kernel's LDS cycles,
//    profiles/pmc_rbt_8192.txt);
//  * f64 MFMA operand maps (cdna_hip_programming.md §3): A lane l holds
//    A[l&15][k=l>>4], B lane l holds B[k=l>>4][l&15], C/D register r of lane l
//    is C[row=(l>>4)+4r][col=l&15] (NOT the f32 C/D map);
//  * C is read into the accumulators up front and written back once;
//  * tiles are dealt to XCDs in contiguous runs (consecutive tiles share an
//    A row panel -> same L2); GELIM_DGEMM_GROUP=g deals a grouped order
//    instead (runs of g tile rows, column-major inside a run) -- measured
//    within noise for g = 4, 8, 16 (profiles/dgemm_r3_lds.txt).
// Interior tiles use 16-byte loads with no bounds logic; edge tiles clamp
// rows/columns (results outside C are never stored) and zero k >= K.
// Contract (checked on the host): A and B 16-byte aligned, lda / ldb / K
// even, ldb > N when N is odd.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
int dgemm_thin(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
               int64_t N, int64_t K, double alpha, int accumulate, int variant, hipStream_t s);

namespace {

constexpr int BM = 128, BN = 128, BK = 16;  // the default (large) tile
constexpr int kThreads = 256;
constexpr int SA = BM + 16, SB = BN + 16;   // LDS row strides (doubles) of the large tile

// Tile geometry: T x T workgroup tile (T = 128, or 64 for thin problems whose
// 128-tiles would leave most CUs idle -- the in-panel K = 32 updates of the
// wide-panel LU, e.g. 8192 x 224), 2 x 2 waves of (T/2) x (T/2).
template <int T>
struct Geo {
  static_assert(T == 128 || T == 64, "tile: 128 or 64");
  static constexpr int TM = T, TN = T;
  static constexpr int SA = T + 16, SB = T + 16;
  static constexpr int WM = T / 2, WN = T / 2;
  static constexpr int MB = WM / 16, NB = WN / 16;
  static constexpr int kCA = T * BK / 2 / kThreads, kCB = BK * T / 2 / kThreads;
  static constexpr int kLds = 2 * BK * SA + 2 * BK * SB;
};

struct Args {
  double* C;
  int64_t ldc;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  int M, N, K;
  int tiles_n, ntiles;
  double alpha;
  int acc;  // 1: C += alpha A B, 0: C = alpha A B (C is not read)
  int group;  // tile order: runs of `group` tile rows, column-major inside a run (<= 1: row-major)
  // column-block-major B / C (0: plain row-major): columns [128 c, 128 c + 128)
  // of the operand live in their own slab at +c * bbs (cbs) doubles, rows at
  // ldb (ldc) inside it -- DistributedRBT's local storage, where every 128-
  // column block is contiguous so its column goes out in one in-place broadcast
  int64_t bbs, cbs;
};

// Column-block-major operands: shift B and C to the slab of the tile's
// 128-column block (a 128- or 64-wide tile never straddles two), so the
// row-major addressing below is unchanged.
__device__ __forceinline__ Args slab_args(const Args& g, int n0) {
  Args s = g;
  const int64_t blk = n0 / 128;
  if (g.bbs) s.B += blk * (g.bbs - 128);
  if (g.cbs) s.C += blk * (g.cbs - 128);
  return s;
}

// Tile index -> (tile row, tile column).  Grouped order: the 64 workgroups an
// XCD runs at once (consecutive indices of its run) cover an 8 x 8 block of
// tiles -- 8 A row panels and 8 B column panels through that XCD's L2 instead
// of 1 A panel and 64 B panels (row-major order).
__device__ __forceinline__ void tile_coords(const Args& g, int tile, int& tr, int& tc) {
  if (g.group <= 1) {
    tr = tile / g.tiles_n;
    tc = tile % g.tiles_n;
    return;
  }
  const int tiles_m = g.ntiles / g.tiles_n, per = g.group * g.tiles_n;
  const int gid = tile / per, first = gid * g.group, l = tile - gid * per;
  const int gs = min(tiles_m - first, g.group);
  tr = first + l % gs;
  tc = l / gs;
}

// 16-byte chunks per thread per tile: A Tx16 -> T*8 chunks, B 16xT -> T*8
template <int T>
struct Stage {
  double2 a[Geo<T>::kCA];
  double2 b[Geo<T>::kCB];
};

template <bool FULL, int T>
__device__ __forceinline__ void load_stage(Stage<T>& st, const Args& g, int m0, int n0, int k0, int t) {
  constexpr int kCA = Geo<T>::kCA, kCB = Geo<T>::kCB;
#pragma unroll
  for (int h = 0; h < kCA; ++h) {
    const int idx = t + kThreads * h;
    const int row = idx >> 3, kc = (idx & 7) * 2;  // 8 chunks per A row of the tile
    if constexpr (FULL) {
      st.a[h] = *reinterpret_cast<const double2*>(g.A + (int64_t)(m0 + row) * g.lda + k0 + kc);
    } else {
      // rows past M are clamped (their products are never stored); K is even,
      // so a chunk is wholly inside or wholly past K
      const int r = min(m0 + row, g.M - 1);
      const int k = k0 + kc;
      const double2 v = *reinterpret_cast<const double2*>(g.A + (int64_t)r * g.lda + min(k, g.K - 2));
      st.a[h] = k < g.K ? v : make_double2(0.0, 0.0);
    }
  }
#pragma unroll
  for (int h = 0; h < kCB; ++h) {
    const int idx = t + kThreads * h;
    const int kr = idx >> (T == 128 ? 6 : 5), nc = (idx & (T / 2 - 1)) * 2;  // T/2 chunks per B row of the tile
    if constexpr (FULL) {
      st.b[h] = *reinterpret_cast<const double2*>(g.B + (int64_t)(k0 + kr) * g.ldb + n0 + nc);
    } else {
      // columns past N are clamped to the last chunk (never stored); with N
      // odd that chunk reads one double of row padding (ldb > N, checked)
      const int k = k0 + kr;
      const int c = min(n0 + nc, (g.N - 1) & ~1);
      const double2 v = *reinterpret_cast<const double2*>(g.B + (int64_t)min(k, g.K - 1) * g.ldb + c);
      st.b[h] = k < g.K ? v : make_double2(0.0, 0.0);
    }
  }
}

template <int T>
__device__ __forceinline__ void store_stage(const Stage<T>& st, double* As, double* Bs, double alpha, int t) {
  constexpr int kCA = Geo<T>::kCA, kCB = Geo<T>::kCB, SA_ = Geo<T>::SA, SB_ = Geo<T>::SB;
#pragma unroll
  for (int h = 0; h < kCA; ++h) {
    const int idx = t + kThreads * h;
    const int row = idx >> 3, kc = (idx & 7) * 2;
    // XOR swizzle: element (k, m) lives at column m ^ (k & 14), so the 8
    // k-chunks of one row that a 16-lane store group holds land on 8
    // distinct bank pairs instead of one (8-way -> conflict-free)
    As[kc * SA_ + (row ^ kc)] = alpha * st.a[h].x;
    As[(kc + 1) * SA_ + (row ^ kc)] = alpha * st.a[h].y;
  }
#pragma unroll
  for (int h = 0; h < kCB; ++h) {
    const int idx = t + kThreads * h;
    const int kr = idx >> (T == 128 ? 6 : 5), nc = (idx & (T / 2 - 1)) * 2;
    *reinterpret_cast<double2*>(&Bs[kr * SB_ + nc]) = st.b[h];
  }
}

// One T x T tile by the 256 threads t = 0..255 (4 waves) over the LDS
// double buffer at lds.  store = false: computed, not written (a persistent
// workgroup's idle half, which still has to meet every barrier).
template <bool FULL, int T = 128>
__device__ __forceinline__ void tile_body(const Args& g0, int m0, int n0, double* lds, int t, bool store = true) {
  const Args g = slab_args(g0, n0);
  using G = Geo<T>;
  constexpr int SA = G::SA, SB = G::SB, WM = G::WM, WN = G::WN, MB = G::MB, NB = G::NB;
  // stage b of the double buffer as offsets from lds (an array of the two
  // pointers indexed at run time lost the LDS address space: every fragment
  // read became a flat load counted in vmcnt, so each k-tile's first wait
  // also drained the next tile's global prefetch)
  auto As = [&](int b) { return lds + b * (BK * SA); };
  auto Bs = [&](int b) { return lds + 2 * BK * SA + b * (BK * SB); };
  const int lane = t & 63, wave = t >> 6;
  const int wm = (wave >> 1) * WM, wn = (wave & 1) * WN;
  const int r16 = lane & 15, q = lane >> 4;

  // the first stage's loads go out before C's, so its LDS store waits only
  // for them (vmcnt is in order)
  Stage<T> st;
  load_stage<FULL, T>(st, g, m0, n0, 0, t);
  dev::d4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + wn + 16 * j + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + q + 4 * r;
        // edge tiles: clamped address, the value is never stored back
        acc[i][j][r] = g.acc ? g.C[(int64_t)(FULL ? row : min(row, g.M - 1)) * g.ldc + (FULL ? col : min(col, g.N - 1))]
                           : 0.0;
      }
    }

  store_stage<T>(st, As(0), Bs(0), g.alpha, t);
  __syncthreads();
  const int nk = (g.K + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage<FULL, T>(st, g, m0, n0, (kt + 1) * BK, t);
    const double* a_s = As(cur) + wm;
    const double* b_s = Bs(cur) + wn + r16;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int k = kk + q;
      const int ac = k * SA + (r16 ^ (k & 14));  // the swizzled column of A(m = .. + r16, k)
      double af[MB], bf[NB];
#pragma unroll
      for (int i = 0; i < MB; ++i) af[i] = a_s[ac + 16 * i];
#pragma unroll
      for (int j = 0; j < NB; ++j) bf[j] = b_s[k * SB + 16 * j];
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_stage<T>(st, As(cur ^ 1), Bs(cur ^ 1), g.alpha, t);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = n0 + wn + 16 * j + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm + 16 * i + q + 4 * r;
        if (store && (FULL || (row < g.M && col < g.N))) {
          g.C[(int64_t)row * g.ldc + col] = acc[i][j][r];
        }
      }
    }
}

template <int T>
__global__ __launch_bounds__(kThreads, 2) void dgemm_kernel(Args g) {
  __shared__ __attribute__((aligned(16))) double lds[Geo<T>::kLds];
  // XCD-aware bijective remap: XCD x (blocks x, x+8, ...) gets a contiguous
  // run of tiles, so tiles sharing an A row panel share that XCD's L2
  const int orig = blockIdx.x;
  const int q = g.ntiles / 8, rem = g.ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  int tr, tc;
  tile_coords(g, tile, tr, tc);
  const int m0 = tr * T, n0 = tc * T;
  if (m0 + T <= g.M && n0 + T <= g.N && (g.K % BK) == 0)
    tile_body<true, T>(g, m0, n0, lds, threadIdx.x);
  else
    tile_body<false, T>(g, m0, n0, lds, threadIdx.x);
}

// Two independent products in ONE launch (the block-LDU engine's pairs of
// thin updates on its critical stream: a block column and a block row that
// read the same operands and write disjoint parts of the matrix): tiles
// [0, g1.ntiles) are g1's, the rest g2's, dealt to XCDs as one range.
template <int T>
__global__ __launch_bounds__(kThreads, 2) void dgemm2_kernel(Args g1, Args g2) {
  __shared__ __attribute__((aligned(16))) double lds[Geo<T>::kLds];
  const int total = g1.ntiles + g2.ntiles;
  const int orig = blockIdx.x;
  const int q = total / 8, rem = total % 8, xcd = orig % 8;
  const int t0 = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  const bool second = t0 >= g1.ntiles;
  const Args g = second ? g2 : g1;
  const int tile = second ? t0 - g1.ntiles : t0;
  int tr, tc;
  tile_coords(g, tile, tr, tc);
  const int m0 = tr * T, n0 = tc * T;
  if (m0 + T <= g.M && n0 + T <= g.N && (g.K % BK) == 0)
    tile_body<true, T>(g, m0, n0, lds, threadIdx.x);
  else
    tile_body<false, T>(g, m0, n0, lds, threadIdx.x);
}

// Persistent form for a grid capped below the CU count (the lookahead side
// stream of plan.hip enqueue_big, which must leave CUs free for the leaf
// chain): 512 threads = two tile engines (2 waves per SIMD, as two of the
// workgroups above), 2 x 72 KiB of LDS, so one workgroup per CU and a grid
// of G workgroups occupies at most G CUs.  Tile pairs are dealt to XCDs in
// contiguous runs (G a multiple of 8); an odd last tile leaves one half
// computing a clamped tile it does not store.
constexpr int kPThreads = 2 * kThreads;
constexpr size_t kStageBytes = sizeof(double) * (2 * BK * SA + 2 * BK * SB);

__global__ __launch_bounds__(kPThreads, 1) void dgemm_persist_kernel(Args g) {
  extern __shared__ __attribute__((aligned(16))) double plds[];
  const int half = __builtin_amdgcn_readfirstlane(threadIdx.x / kThreads), t = threadIdx.x % kThreads;
  double* lds = plds + half * (kStageBytes / sizeof(double));
  const int npairs = (g.ntiles + 1) / 2;
  const int xcd = blockIdx.x % 8, local = blockIdx.x / 8, per = gridDim.x / 8;
  const int q = npairs / 8, rem = npairs % 8;
  const int beg = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
  const int end = beg + q + (xcd < rem ? 1 : 0);
  for (int pr = beg + local; pr < end; pr += per) {
    const int tile0 = 2 * pr + half;
    const bool store = tile0 < g.ntiles;
    const int tile = store ? tile0 : g.ntiles - 1;
    int tr, tc;
    tile_coords(g, tile, tr, tc);
    const int m0 = tr * BM, n0 = tc * BN;
    // an opaque copy of t per pair: nothing thread-dependent is hoisted out
    // of the loop (hoisted address terms pushed the body past 256 VGPRs)
    int tt = t;
    asm volatile("" : "+v"(tt));
    if (m0 + BM <= g.M && n0 + BN <= g.N && (g.K % BK) == 0)
      tile_body<true, 128>(g, m0, n0, lds, tt, store);
    else
      tile_body<false, 128>(g, m0, n0, lds, tt, store);
    __syncthreads();  // the next pair's first stage overwrites this one's LDS
  }
}

}  // namespace

// C (M x N, ldc) += alpha * A (M x K, lda) * B (K x N, ldb); alpha in {+1, -1}
// in practice (any value works: A is scaled once on its way into LDS).
// group < 0: row-major tile order (grouped orders 4 / 8 / 16 measured within
// noise of it, profiles/dgemm_r3_lds.txt), else that order.  C is stored
// plainly (write-through stores were within noise, profiles/dgemm_wt_r4.txt).
int dgemm_launch(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate, int group_arg,
                 int64_t bbs = 0, int64_t cbs = 0) {
  if (M <= 0 || N <= 0 || K <= 0) return GELIM_OK;
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX) return GELIM_FAIL(GELIM_E_ARG, "dgemm: dimension > 2^31");
  // column-block-major operands: whole 128-column blocks, 128-wide slabs
  if ((bbs || cbs) && (N % 128 || (bbs && (ldb < 128 || bbs < ldb * K || (bbs & 1))) ||
                       (cbs && (ldc < 128 || cbs < ldc * M))))
    return GELIM_FAIL(GELIM_E_ARG, "dgemm: column-block-major operands need N % 128 == 0 and 128-wide slabs");
  const int64_t nb_row = bbs ? std::min<int64_t>(N, 128) : N, nc_row = cbs ? std::min<int64_t>(N, 128) : N;
  // 16-byte operand chunks: 16-byte aligned A and B, even leading dimensions
  // and K, and one double of row padding in B when N is odd
  if ((K & 1) || (lda & 1) || (ldb & 1) || (((uintptr_t)A | (uintptr_t)B) & 15) || ((N & 1) && ldb <= N) ||
      lda < K || ldb < nb_row || ldc < nc_row)
    return GELIM_FAIL(GELIM_E_ARG, "dgemm: unsupported alignment / leading dimensions (K=" + std::to_string(K) +
                                       " lda=" + std::to_string(lda) + " ldb=" + std::to_string(ldb) + ")");
  const int tm = (int)((M + BM - 1) / BM), tn = (int)((N + BN - 1) / BN);
  const int group = group_arg >= 0 ? group_arg : 1;
  Args g{C, ldc, A, lda, B, ldb, (int)M, (int)N, (int)K, tn, tm * tn, alpha, accumulate ? 1 : 0, group, bbs, cbs};
  // max_wg > 0: at most max_wg CUs (rounded down to a multiple of 8)
  const int cap = max_wg > 0 ? std::max(8, max_wg / 8 * 8) : 0;
  // few tiles: one 256-thread workgroup per tile already stays within the
  // cap (<= tiles CUs) and halves the per-workgroup work
  if (cap > 0 && tm * tn > cap) {
    static const bool attr = [] {
      return hipFuncSetAttribute((const void*)dgemm_persist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)(2 * kStageBytes)) == hipSuccess;
    }();
    if (!attr) return GELIM_FAIL(GELIM_E_HIP, "dgemm: 144 KiB of LDS per workgroup refused");
    const int grid = std::min(cap, (tm * tn + 1) / 2 + 7) / 8 * 8;  // whole XCD rounds
    hipLaunchKernelGGL(dgemm_persist_kernel, dim3((unsigned)std::max(grid, 8)), dim3(kPThreads), 2 * kStageBytes, s,
                       g);
  } else {
    // thin problems (fewer 128-tiles than CUs, e.g. the
    // in-panel K = 32 updates, 8192 x 224): 64-tiles, 4x the workgroups
    static const int ncu = [] {
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      return cus;
    }();
    // (the register-direct thin kernel of dgemm_thin.hip measured no faster
    // at the block-LDU engine's K = 128 / 256 shapes, profiles/dgemm_thin_r4.txt;
    // it stays callable as gelim_gpu_dgemm_thin)
    const bool small = (int64_t)tm * tn < (int64_t)ncu;
    // (capped: 64-tiles too when their grid stays within the cap)
    const int64_t t64 = ((M + 63) / 64) * ((N + 63) / 64);
    if (small && (cap == 0 || t64 <= cap)) {
      const int tm6 = (int)((M + 63) / 64), tn6 = (int)((N + 63) / 64);
      Args g6 = g;
      g6.tiles_n = tn6;
      g6.ntiles = tm6 * tn6;
      hipLaunchKernelGGL(dgemm_kernel<64>, dim3((unsigned)(tm6 * tn6)), dim3(kThreads), 0, s, g6);
    } else {
      hipLaunchKernelGGL(dgemm_kernel<128>, dim3((unsigned)(tm * tn)), dim3(kThreads), 0, s, g);
    }
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int dgemm_capped(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate = 1) {
  return dgemm_launch(C, ldc, A, lda, B, ldb, M, N, K, alpha, max_wg, s, accumulate, -1);
}

int dgemm(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
          int64_t N, int64_t K, double alpha, hipStream_t s) {
  return dgemm_capped(C, ldc, A, lda, B, ldb, M, N, K, alpha, 0, s);
}

// C = alpha * A * B (accumulate = 0: C is written, never read) or C += ...
int dgemm_ex(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
             int64_t N, int64_t K, double alpha, int accumulate, hipStream_t s) {
  return dgemm_capped(C, ldc, A, lda, B, ldb, M, N, K, alpha, 0, s, accumulate);
}

// K = 128 products as one 64-thread workgroup per 16 x 16 tile of C: for
// the 128-wide products on a latency-bound chain (the randomised engines'
// W = Dinv A_k,rest and block-column / block-row updates).  Those have few
// 64-tiles, so a 64-tile grid leaves most CUs idle, and each of its
// workgroups needs 40 KB of LDS -- beside a bulk GEMM whose 128-tiles hold
// 2 x 72 KB of every CU's LDS it cannot start until side workgroups retire
// (28.8 us for 128 x 8064 x 128 under the hip-rbt side update,
// profiles/rbt_trace_8192_r6.txt).  A tile workgroup pulls ~32 KB (16 rows of
// A, a 16-column strip of B) and uses no LDS: each lane loads its own MFMA
// fragments, all in flight before the first MFMA (A: 16 rows x 4 k per
// instruction; B: 4 rows x 128 B), then 32 v_mfma_f64_16x16x4f64 over k =
// 0..127 in order, A scaled by alpha on its way in, C read first -- the tile
// kernel's per-element operation order, so the bits are dgemm's
// (tests/test_gpu_dist_rbt.py::test_chain_products_match_dgemm).  128 x 128
// x 128: 3.9 us against 8.6 for the 64-tile grid
// (profiles/dist_rbt_replay_r6.md).  At 128 x 8000 the tiles' operand
// traffic (4x the 64-tiles') lost more than the LDS wait cost: hip-rbt keeps
// dgemm there (profiles/rbt_trace_8192_r6.txt).
struct Tile16 {
  double* C;
  int64_t ldc;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  int nt;  // 16-column tiles of C
};

template <bool kAcc>
__global__ __launch_bounds__(64) void tile16_kernel(Tile16 o0, Tile16 o1, int n0, double alpha) {
  const int lane = threadIdx.x, r16 = lane & 15, q = lane >> 4;
  int b = blockIdx.x;
  const Tile16 o = b < n0 ? o0 : o1;
  b = b < n0 ? b : b - n0;
  const int tm = b / o.nt, tn = b % o.nt;
  const double* Ab = o.A + (int64_t)(16 * tm + r16) * o.lda + q;
  const double* Bb = o.B + (int64_t)q * o.ldb + 16 * tn + r16;
  double av[32], bv[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    av[s] = Ab[4 * s];
    bv[s] = Bb[(int64_t)(4 * s) * o.ldb];
  }
  double* Ct = o.C + (int64_t)(16 * tm) * o.ldc + 16 * tn;
  dev::d4 acc = {0.0, 0.0, 0.0, 0.0};
  if (kAcc) {
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = Ct[(int64_t)(q + 4 * r) * o.ldc + r16];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < 32; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(alpha * av[s], bv[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) Ct[(int64_t)(q + 4 * r) * o.ldc + r16] = acc[r];
}

// Up to two independent K = 128 products C (+)= alpha A B in one launch of
// 16 x 16 tiles (M, N multiples of 16; an op with M or N <= 0 is skipped).
int dgemm_tiles(const GemmOp& p1, const GemmOp& p2, double alpha, int accumulate, hipStream_t s) {
  const GemmOp* ops[2] = {&p1, &p2};
  Tile16 t[2] = {};
  int n[2] = {0, 0};
  for (int i = 0; i < 2; ++i) {
    const GemmOp& o = *ops[i];
    if (o.M <= 0 || o.N <= 0) continue;
    if (o.K != 128 || o.M % 16 || o.N % 16 || o.lda < 128 || o.ldb < o.N || o.ldc < o.N ||
        (o.M / 16) * (o.N / 16) > INT32_MAX / 2)
      return GELIM_FAIL(GELIM_E_ARG, "dgemm_tiles: K must be 128, M and N multiples of 16");
    t[i] = Tile16{o.C, o.ldc, o.A, o.lda, o.B, o.ldb, (int)(o.N / 16)};
    n[i] = (int)((o.M / 16) * (o.N / 16));
  }
  if (n[0] + n[1] == 0) return GELIM_OK;
  if (n[0] == 0) {  // op 0 empty: op 1 alone
    t[0] = t[1];
    n[0] = n[1];
    n[1] = 0;
  }
  const dim3 grid((unsigned)(n[0] + n[1]));
  if (accumulate)
    hipLaunchKernelGGL(tile16_kernel<true>, grid, dim3(64), 0, s, t[0], t[1], n[0], alpha);
  else
    hipLaunchKernelGGL(tile16_kernel<false>, grid, dim3(64), 0, s, t[0], t[1], n[0], alpha);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Two independent C += alpha A B products (same alpha / accumulate) in one
// launch (dgemm2_kernel); either may be empty.  Same operand contract as
// dgemm_launch.
int dgemm_pair(const GemmOp& p1, const GemmOp& p2, double alpha, int accumulate, hipStream_t s) {
  const GemmOp* ops[2] = {&p1, &p2};
  for (const GemmOp* o : ops) {
    if (o->M <= 0 || o->N <= 0 || o->K <= 0) continue;
    if (o->M > INT32_MAX || o->N > INT32_MAX || o->K > INT32_MAX)
      return GELIM_FAIL(GELIM_E_ARG, "dgemm_pair: dimension > 2^31");
    if ((o->K & 1) || (o->lda & 1) || (o->ldb & 1) || (((uintptr_t)o->A | (uintptr_t)o->B) & 15) ||
        ((o->N & 1) && o->ldb <= o->N) || o->lda < o->K || o->ldb < o->N || o->ldc < o->N)
      return GELIM_FAIL(GELIM_E_ARG, "dgemm_pair: unsupported alignment / leading dimensions");
  }
  const bool e1 = p1.M <= 0 || p1.N <= 0 || p1.K <= 0, e2 = p2.M <= 0 || p2.N <= 0 || p2.K <= 0;
  if (e1 && e2) return GELIM_OK;
  if (e1) return dgemm_ex(p2.C, p2.ldc, p2.A, p2.lda, p2.B, p2.ldb, p2.M, p2.N, p2.K, alpha, accumulate, s);
  if (e2) return dgemm_ex(p1.C, p1.ldc, p1.A, p1.lda, p1.B, p1.ldb, p1.M, p1.N, p1.K, alpha, accumulate, s);
  static const int ncu = [] {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus;
  }();
  auto args = [&](const GemmOp& o, int T) {
    const int tm = (int)((o.M + T - 1) / T), tn = (int)((o.N + T - 1) / T);
    return Args{o.C, o.ldc, o.A, o.lda, o.B, o.ldb, (int)o.M, (int)o.N, (int)o.K, tn, tm * tn, alpha,
                accumulate ? 1 : 0, 1, 0, 0};
  };
  const Args a1 = args(p1, 128), a2 = args(p2, 128);
  if ((int64_t)a1.ntiles + a2.ntiles < (int64_t)ncu) {  // thin: 64-tiles, as dgemm_launch
    const Args b1 = args(p1, 64), b2 = args(p2, 64);
    hipLaunchKernelGGL(dgemm2_kernel<64>, dim3((unsigned)(b1.ntiles + b2.ntiles)), dim3(kThreads), 0, s, b1, b2);
  } else {
    hipLaunchKernelGGL(dgemm2_kernel<128>, dim3((unsigned)(a1.ntiles + a2.ntiles)), dim3(kThreads), 0, s, a1, a2);
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace gelim

extern "C" int gelim_gpu_dgemm(double* dC, int64_t ldc, const double* dA, int64_t lda, const double* dB,
                               int64_t ldb, int64_t M, int64_t N, int64_t K, double alpha, void* stream) {
  return gelim::dgemm(dC, ldc, dA, lda, dB, ldb, M, N, K, alpha, (hipStream_t)stream);
}

// an explicit tile order (runs of `group` tile rows; tests of the grouped order)
extern "C" int gelim_gpu_dgemm_grouped(double* dC, int64_t ldc, const double* dA, int64_t lda, const double* dB,
                                       int64_t ldb, int64_t M, int64_t N, int64_t K, double alpha, int max_wg,
                                       int group, void* stream) {
  return gelim::dgemm_launch(dC, ldc, dA, lda, dB, ldb, M, N, K, alpha, max_wg, (hipStream_t)stream, 1,
                             group < 0 ? 0 : group);
}

// Column-block-major B and / or C (bbs / cbs: doubles between consecutive
// 128-column slabs; 0 = plain row-major): C (+)= alpha A B with N a multiple
// of 128.  DistributedRBT's local storage (parallel/dist_rbt.py).
extern "C" int gelim_gpu_dgemm_bm(double* dC, int64_t ldc, int64_t cbs, const double* dA, int64_t lda,
                                  const double* dB, int64_t ldb, int64_t bbs, int64_t M, int64_t N, int64_t K,
                                  double alpha, int accumulate, int max_wg, void* stream) {
  return gelim::dgemm_launch(dC, ldc, dA, lda, dB, ldb, M, N, K, alpha, max_wg, (hipStream_t)stream, accumulate, -1,
                             bbs, cbs);
}

// the persistent form on at most max_wg CUs (tests / benchmarks)
extern "C" int gelim_gpu_dgemm_capped(double* dC, int64_t ldc, const double* dA, int64_t lda, const double* dB,
                                      int64_t ldb, int64_t M, int64_t N, int64_t K, double alpha, int max_wg,
                                      void* stream) {
  return gelim::dgemm_capped(dC, ldc, dA, lda, dB, ldb, M, N, K, alpha, max_wg, (hipStream_t)stream);
}
