// Wide-panel blocked LU for large systems (n > 2048): the kernels.
//
// What it computes: the reference's forward elimination with partial
// pivoting (getPivot + computeGauss, OpenMP_and_MPI/gauss_openmp/
// gauss_external_input.c:123-182; the external programs accept any n,
// Pthreads/Version-1/gauss_external_input.c:34-86, e.g. memplus at
// n = 17758), as a right-looking LU with LAPACK row order: outer panels of
// nb = 256 columns, each factored as 32-column leaves; the driver is in
// plan.hip (big_factor).
//
// Why a multi-workgroup leaf: the register-resident panels of lu_panel.hip /
// rlu.hip keep an m x 16 panel on ONE CU, which caps m at 2048 (256 KiB of
// VGPRs).  Past that the panel had to shrink to 8/4/2 columns and the
// trailing update became a bandwidth-bound rank-2..8 update.  Here a leaf of
// m x 32 is spread over P participant workgroups of NWV waves each (4 rows x
// 32 columns per lane, one wave per SIMD: 256 NWV rows per workgroup), every
// column's pivot is an exact global arg-max (ties to the lowest row, like the
// reference's strict '>'), and the trailing update of each outer panel is
// one fp64 MFMA GEMM with K = nb (dgemm.hip) instead of rank-2 sweeps.  The
// leaf kernel itself is in leaf.h (instantiated by leaf_w*.hip); this file
// holds the row-movement, TRSM and back-substitution kernels around it and
// the host entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <utility>

#include "device_common.h"
#include "gelim/internal.h"
#include "leaf.h"

namespace gelim {
namespace big {
namespace {

using leafk::LW;

// ---- row interchanges for the other columns + TRSM of a leaf's U rows -----
// One thread per column of [lbeg, lend) (interchanges only: the L part left
// of the leaf) and of [rbeg, rend) (interchanges, then -- for columns below
// trsm_end -- U12 = L11^-1 A12 on the LW rows starting at row c0, L11 being
// the leaf at (c0, c0)).  A points at row c0, column 0; rows of the pair
// list are relative to c0 (pairs == nullptr: no interchanges).  Every
// touched source row is read before any destination is written (the pair
// list is a permutation of <= 2 LW rows).
//
// The driver uses it twice per leaf: right after the leaf (interchanges on
// every other column, TRSM only inside the outer panel), and once the whole
// outer panel is factored (no interchanges, TRSM of the leaf's rows of the
// columns right of the panel).  Updating those columns any earlier would mix
// rows that carry a leaf's update with rows that do not when a later leaf
// swaps rows across the panel boundary.
constexpr int kSwThreads = 64;  // one wave per workgroup: one CU per 64 columns

struct SwapArgs {
  double* A;
  int64_t lda;
  int c0, lbeg, lend, rbeg, rend, trsm_end, nrows;
  const int* pairs;
  const double* L;  // L11 (unit lower, LW x LW) of the TRSM, leading dimension ldl
  int64_t ldl;
};

__global__ __launch_bounds__(kSwThreads) void laswp_trsm_kernel(SwapArgs g) {
  __shared__ double sLt[LW][LW];        // transposed L11: sLt[i][j] = L[j][i]
  __shared__ double xs[LW][kSwThreads];
  __shared__ int sdst[2 * LW];          // validated pair list (dst -1: none)
  const int lane = threadIdx.x;
  const int64_t lda = g.lda;
  // one round trip for everything the columns depend on: lane e holds pair
  // e (dst, src) -- read back with readlane, so row offsets are scalar --
  // and 16 elements of L11 (every load unconditional, issued together)
  int cnt = 0, pd = -1, ps = -1;
  if (g.pairs != nullptr) {
    cnt = min(g.pairs[0], 2 * LW);
    pd = g.pairs[1 + 2 * lane];
    ps = g.pairs[2 + 2 * lane];
  }
  double lv[LW * LW / kSwThreads];
#pragma unroll
  for (int k = 0; k < LW * LW / kSwThreads; ++k) {
    const int e = lane + kSwThreads * k;
    lv[k] = g.L[(int64_t)(e / LW) * g.ldl + (e % LW)];
  }
  const bool pok = lane < cnt && pd >= 0 && pd < g.nrows && ps >= 0 && ps < g.nrows;
  pd = pok ? pd : -1;
  ps = pok ? ps : 0;
  // destinations are read after lanes have diverged: from LDS, never with
  // readlane (a lane that has left keeps a stale register, and the select
  // above may be sunk past the divergence)
  sdst[lane] = pd;
#pragma unroll
  for (int k = 0; k < LW * LW / kSwThreads; ++k) {
    const int e = lane + kSwThreads * k;
    sLt[e % LW][e / LW] = lv[k];
  }
  const int nleft = g.lend - g.lbeg, nright = g.rend - g.rbeg;
  const int idx = blockIdx.x * kSwThreads + lane;
  const bool any = idx < nleft + nright;
  const bool right = idx >= nleft;
  const int c = any ? (right ? idx - nleft + g.rbeg : g.lbeg + idx) : 0;
  double* col = g.A + c;
  const bool trsm = any && right && c < g.trsm_end;
  // gathers: every touched source row, before any destination is written
  double gsrc[2 * LW];
#pragma unroll
  for (int e = 0; e < 2 * LW; ++e) gsrc[e] = col[(int64_t)__builtin_amdgcn_readlane(ps, e) * lda];
  double x[LW];
  if (__ballot(trsm) != 0) {
#pragma unroll
    for (int j = 0; j < LW; ++j) x[j] = col[(int64_t)j * lda];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // sLt written (single-wave workgroup)
  if (!any) return;
  if (!trsm) {
#pragma unroll
    for (int e = 0; e < 2 * LW; ++e) {
      const int d = sdst[e];
      if (d >= 0) col[(int64_t)d * lda] = gsrc[e];
    }
    return;
  }
  // top LW rows of the column after the interchanges: staged through LDS
  // (the destination row is uniform, the register array is not indexable)
#pragma unroll
  for (int j = 0; j < LW; ++j) xs[j][lane] = x[j];
#pragma unroll
  for (int e = 0; e < 2 * LW; ++e) {
    const int d = sdst[e];
    if (d >= 0) {
      if (d < LW) xs[d][lane] = gsrc[e];
      else col[(int64_t)d * lda] = gsrc[e];
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < LW; ++j) x[j] = xs[j][lane];
  // forward substitution, column i of L read (uniform, 16-byte LDS reads)
  // one step ahead of its use
  double lc[LW];
#pragma unroll
  for (int j = 1; j < LW; ++j) lc[j] = sLt[0][j];
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    double ln[LW];
    if (i + 1 < LW) {
#pragma unroll
      for (int j = i + 2; j < LW; ++j) ln[j] = sLt[i + 1][j];
    }
    __builtin_amdgcn_sched_barrier(0);
    const double xi = x[i];
    col[(int64_t)i * lda] = xi;
#pragma unroll
    for (int j = i + 1; j < LW; ++j) x[j] = fma(-lc[j], xi, x[j]);
#pragma unroll
    for (int j = i + 2; j < LW; ++j) lc[j] = ln[j];
  }
}

// ---- a whole outer panel's interchanges on other columns ---------------------
// The lookahead schedule (plan.hip) applies an outer panel's row movement to
// the columns it does not own -- the L part left of the panel and the
// trailing columns the side stream updates -- in ONE launch: per column, the
// panel's leaf pair lists in order (each a permutation of <= 2 LW rows:
// every source gathered before any destination is written).  The lists are
// wave-uniform, so their words are scalar loads (no LDS, no readlane).
struct PanelSwapArgs {
  double* A;          // row 0, column 0 of the system
  int64_t lda;
  int n;              // rows of the system (list entries are validated against it)
  int c0;             // diagonal of the panel's first leaf
  int nleaves;
  const int* pairs;   // nleaves slots of `slot` ints: [0] count, then (dst, src) relative to the leaf's diagonal
  int slot;
  int lbeg, lend, rbeg, rend;  // columns [lbeg, lend) and [rbeg, rend)
};

__device__ __forceinline__ void laswp_panel_block(const PanelSwapArgs& g, int idx, int nl, int nr) {
  const bool any = idx < nl + nr;
  // lanes past the ranges read a valid column and store nothing (no early
  // exit: the loop below stays uniform)
  const int c = any ? (idx < nl ? g.lbeg + idx : g.rbeg + idx - nl) : (nl > 0 ? g.lbeg : g.rbeg);
  double* col = g.A + c;
#pragma unroll 1
  for (int l = 0; l < g.nleaves; ++l) {
    const int* pr = g.pairs + (int64_t)l * g.slot;
    const int cnt = min(pr[0], 2 * LW);
    const int base = g.c0 + l * LW;
    double v[2 * LW];
#pragma unroll
    for (int e = 0; e < 2 * LW; ++e) {
      const int src = base + pr[2 + 2 * e];
      const bool ok = e < cnt && src >= base && src < g.n;
      v[e] = col[(int64_t)(ok ? src : base) * g.lda];
    }
#pragma unroll
    for (int e = 0; e < 2 * LW; ++e) {
      const int dst = base + pr[1 + 2 * e], src = base + pr[2 + 2 * e];
      if (any && e < cnt && dst >= base && dst < g.n && src >= base && src < g.n) col[(int64_t)dst * g.lda] = v[e];
    }
  }
}

__global__ __launch_bounds__(64) void laswp_panel_kernel(PanelSwapArgs g) {
  const int nl = g.lend - g.lbeg, nr = g.rend - g.rbeg;
  // grid-stride over 64-column blocks (a capped grid on the lookahead side
  // stream); the block index is wave-uniform, so the loop is too
  for (int blk = blockIdx.x; blk * 64 < nl + nr; blk += gridDim.x)
    laswp_panel_block(g, blk * 64 + threadIdx.x, nl, nr);
}

// ---- an outer panel's row movement as ONE permutation -------------------------
// laswp_panel replays the leaves' lists one after another per column (a chain
// of dependent gathers: ~90 us whatever the width).  Composed once, the
// panel's movement is a single permutation of <= 64 rows per leaf, applied
// by a plain gather-then-scatter over (row, column) tiles.
//
// compose: one workgroup folds the nleaves pair lists (rows relative to
// each leaf's diagonal c0 + 32 l) into the net list {count, (dst, src)...}
// of rows relative to c0.  LDS holds, for every row position of the panel's
// m rows, the original row now sitting there.
struct ComposeArgs {
  int m;              // rows from c0 to the end of the system
  int nleaves;
  const int* pairs;   // nleaves slots of `slot` ints
  int slot;
  int* net;           // [0] = count, then (dst, src) relative to c0
};
constexpr int kCmpThreads = 1024;

__global__ __launch_bounds__(kCmpThreads) void compose_kernel(ComposeArgs g) {
  extern __shared__ int content[];  // [m] + 1 counter
  const int t = threadIdx.x;
  for (int i = t; i < g.m; i += kCmpThreads) content[i] = i;
  if (t == 0) content[g.m] = 0;
  __syncthreads();
  for (int l = 0; l < g.nleaves; ++l) {
    const int* pr = g.pairs + (int64_t)l * g.slot;
    const int cnt = min(pr[0], 2 * LW);
    const int base = l * LW;
    int v = 0, dst = -1;
    if (t < cnt) {
      const int d = base + pr[1 + 2 * t], sr = base + pr[2 + 2 * t];
      if (d >= base && d < g.m && sr >= base && sr < g.m) {
        v = content[sr];
        dst = d;
      }
    }
    __syncthreads();  // every source read before any destination is written
    if (dst >= 0) content[dst] = v;
    __syncthreads();
  }
  for (int i = t; i < g.m; i += kCmpThreads) {
    const int r = content[i];
    if (r != i) {
      const int e = atomicAdd(&content[g.m], 1);
      g.net[1 + 2 * e] = i;
      g.net[2 + 2 * e] = r;
    }
  }
  __syncthreads();
  if (t == 0) g.net[0] = content[g.m];
}

// apply: 16 columns x all moved rows per workgroup, every source value in
// registers (<= 512 rows: 32 per thread) before the barrier, then the
// stores; a grid-stride loop over 16-column chunks of [lbeg, lend) and
// [rbeg, rend).  Workgroups touch disjoint columns, so no cross-workgroup
// ordering is needed.
struct NetSwapArgs {
  double* A;          // row c0, column 0 of the system
  int64_t lda;
  const int* net;
  int lbeg, lend, rbeg, rend;
};
constexpr int kNsCols = 16, kNsThreads = 256, kNsGroups = kNsThreads / kNsCols;
constexpr int kNsPer = 32, kNsMax = kNsGroups * kNsPer;  // 512 rows

__global__ __launch_bounds__(kNsThreads) void laswp_net_kernel(NetSwapArgs g) {
  __shared__ int2 lst[kNsMax];
  const int t = threadIdx.x, cl = t % kNsCols, rg = t / kNsCols;
  const int cnt = min(g.net[0], kNsMax);
  if (cnt <= 0) return;
  for (int e = t; e < cnt; e += kNsThreads) lst[e] = make_int2(g.net[1 + 2 * e], g.net[2 + 2 * e]);
  __syncthreads();
  const int nl = g.lend - g.lbeg, nr = g.rend - g.rbeg;
  const int nch = (nl + nr + kNsCols - 1) / kNsCols;
  for (int ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int idx = ch * kNsCols + cl;
    const bool any = idx < nl + nr;
    const int c = any ? (idx < nl ? g.lbeg + idx : g.rbeg + idx - nl) : (nl > 0 ? g.lbeg : g.rbeg);
    double v[kNsPer];
#pragma unroll
    for (int k = 0; k < kNsPer; ++k) v[k] = g.A[(int64_t)lst[min(rg + k * kNsGroups, cnt - 1)].y * g.lda + c];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every gather landed before any scatter
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kNsPer; ++k) {
      const int e = rg + k * kNsGroups;
      if (any && e < cnt) g.A[(int64_t)lst[e].x * g.lda + c] = v[k];
    }
    __syncthreads();  // (the gathers of the next chunk read other columns; kept for clarity of the LDS list)
  }
}

// ---- U12 of a whole outer panel in one launch --------------------------------
// U12 = L11^-1 A12 for the nb (<= 256, multiple of LW) rows of an outer panel,
// L11 unit lower.  One workgroup per 32 columns keeps its nb x 32 block of
// A12 in LDS for the whole forward substitution: per 32-row block j, the
// diagonal 32x32 solve (lane = column, registers) and the update of the
// rows below (VALU, L staged in LDS, the solved block in registers).  This
// replaces nb/32 alternating launches (32-row TRSM, then a K = 32 GEMM of
// the rows below) -- 15 launches per 256-column panel.
constexpr int kTrNb = 256;                    // max rows
constexpr int kTrCols = 32;                   // columns per workgroup

struct PanelTrsmArgs {
  double* C;          // row 0 of the panel's rows, first column of the range
  int64_t ldc;
  int ncols, nb;
  const double* L;    // L11 (nb x nb, unit lower), leading dimension ldl
  int64_t ldl;
};

constexpr int kTrThreads = 512;                // 16 row groups of 32 columns
constexpr int kTrGroups = kTrThreads / kTrCols;

// one 32-column block [c0, c0 + 32) of the range
__device__ __forceinline__ void panel_trsm_block(const PanelTrsmArgs& g, double (*X)[kTrCols + 1],
                                                 double (*Ls)[LW + 2], int t, int col, int rg, int c0) {
  const bool cok = c0 + col < g.ncols;
  const int nb = g.nb;
  double* cp = g.C + c0 + (cok ? col : 0);
  for (int r = rg; r < nb; r += kTrGroups) X[r][col] = cok ? cp[(int64_t)r * g.ldc] : 0.0;
  for (int j0 = 0; j0 < nb; j0 += LW) {
    for (int e = t; e < (nb - j0) * LW; e += kTrThreads)
      Ls[e / LW][e % LW] = g.L[(int64_t)(j0 + e / LW) * g.ldl + j0 + e % LW];
    __syncthreads();
    if (t < kTrCols) {  // diagonal block, lane = column
      double x[LW];
#pragma unroll
      for (int i = 0; i < LW; ++i) x[i] = X[j0 + i][col];
#pragma unroll
      for (int i = 0; i < LW; ++i)
#pragma unroll
        for (int r = i + 1; r < LW; ++r) x[r] = fma(-Ls[r][i], x[i], x[r]);
#pragma unroll
      for (int i = 0; i < LW; ++i) X[j0 + i][col] = x[i];
    }
    __syncthreads();
    if (j0 + LW < nb) {
      double xj[LW];
#pragma unroll
      for (int i = 0; i < LW; ++i) xj[i] = X[j0 + i][col];
      for (int r = j0 + LW + rg; r < nb; r += kTrGroups) {
        // the row's 32 multipliers: 16 uniform 16-byte LDS reads, then the
        // dot product from registers
        const double2* lr = reinterpret_cast<const double2*>(&Ls[r - j0][0]);
        double l[LW];
#pragma unroll
        for (int i = 0; i < LW / 2; ++i) {
          const double2 v = lr[i];
          l[2 * i] = v.x;
          l[2 * i + 1] = v.y;
        }
        double acc = X[r][col];
#pragma unroll
        for (int i = 0; i < LW; ++i) acc = fma(-l[i], xj[i], acc);
        X[r][col] = acc;
      }
    }
    __syncthreads();
  }
  if (cok)
    for (int r = rg; r < nb; r += kTrGroups) cp[(int64_t)r * g.ldc] = X[r][col];
}

__global__ __launch_bounds__(kTrThreads) void panel_trsm_kernel(PanelTrsmArgs g) {
  extern __shared__ double trsm_lds[];
  double (*X)[kTrCols + 1] = reinterpret_cast<double (*)[kTrCols + 1]>(trsm_lds);                  // [nb][33]
  // L rows [j0, nb) x 32 columns, rows 16-byte aligned (34 doubles)
  double (*Ls)[LW + 2] = reinterpret_cast<double (*)[LW + 2]>(trsm_lds + kTrNb * (kTrCols + 1));
  const int t = threadIdx.x, col = t & 31, rg = t >> 5;
  // grid-stride over 32-column blocks (a capped grid on the lookahead side
  // stream); every loop below ends in a barrier, so X and Ls are free again
  for (int c0 = blockIdx.x * kTrCols; c0 < g.ncols; c0 += gridDim.x * kTrCols)
    panel_trsm_block(g, X, Ls, t, col, rg, c0);
}

// ---- block back substitution helpers ----------------------------------------
// y[i] = A[i][n] - sum_{j >= K} A[i][j] x[j] for the top K rows (x[K..n) is
// the solved tail), bnorm[i] = A[i][n] / A[i][i] (the reference's normalised
// B after elimination).  One wave per row.
__global__ __launch_bounds__(256) void tail_gemv_kernel(const double* __restrict__ A, int64_t lda, int n, int K,
                                                        const double* __restrict__ x, double* __restrict__ y,
                                                        double* __restrict__ bnorm) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= K) return;
  const double* ar = A + (int64_t)row * lda;
  double s = 0.0;
  for (int j = K + lane; j < n; j += 64) s = fma(ar[j], x[j], s);
  s = dev::wave_sum(s);
  if (lane == 0) {
    y[row] = ar[n] - s;
    if (bnorm) bnorm[row] = ar[n] / ar[row];
  }
}

// fold the tail solver's info words into the system's: singular column
// offset by K, hand-off errors kept
__global__ void fold_info_kernel(int* __restrict__ info, const int* __restrict__ tinfo, int K) {
  if (threadIdx.x == 0) {
    if (info[0] == 0 && tinfo[0] != 0) info[0] = K + tinfo[0];
    if (info[1] == 0 && tinfo[1] != 0) info[1] = tinfo[1];
  }
}

}  // namespace

struct LeafShape {
  int nwv, rw;  // waves per participant, rows per lane
};

namespace sleaf {  // leaf_stream.hip
size_t scratch_bytes();
int factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
           void* scratch, hipStream_t s);
}  // namespace sleaf

// the register leaf's exchange areas, then the streamed leaf's scratch
size_t workspace_bytes() { return leafk::kKeyBytes + leafk::kRowBytes + sleaf::scratch_bytes(); }
int leaf_width() { return LW; }

// Leaf participant shape for m rows: one wave of 2 rows per lane (1x2, the
// measured best, profiles/leaf_shape_r4.txt), then 2x2 and 4x4 waves x rows
// per lane as m outgrows kMaxP participants of the smaller shape.  (1x4, 1x1
// and 4x1 were measured and dropped in round 5 with their knobs.)
LeafShape leaf_shape(int64_t m) {
  for (LeafShape sh : {LeafShape{1, 2}, LeafShape{2, 2}})
    if (m <= (int64_t)leafk::kMaxP * 64 * sh.nwv * sh.rw) return sh;
  return LeafShape{4, 4};
}
int leaf_waves(int64_t m) { return leaf_shape(m).nwv; }
// rows of one participant
int64_t participant_rows(LeafShape sh) { return (int64_t)sh.nwv * 64 * sh.rw; }
// Rows the register-resident leaf holds (256 participants x 4 waves x 256
// rows: the chip's register file); taller panels take the streamed leaf
// (leaf_stream.hip, HBM-resident, same results bit for bit), so the leaf
// itself no longer caps the order -- memory does.
int64_t reg_max_rows() { return (int64_t)leafk::kMaxP * 4 * leafk::kRowsPerWave; }
int64_t max_rows() { return (int64_t)1 << 26; }
// GELIM_LEAF_STREAM=1: the streamed leaf at every m (tests compare the two);
// read per call
bool leaf_streamed(int64_t m) {
  if (m > reg_max_rows()) return true;
  const char* e = std::getenv("GELIM_LEAF_STREAM");
  return e != nullptr && std::atoi(e) == 1;
}
int leaf_participants(int64_t m) {
  const int64_t rows = participant_rows(leaf_shape(m));
  return (int)((m + rows - 1) / rows);
}
// CUs a leaf of m rows needs at once (its waves take a whole SIMD's registers:
// four single-wave participants or one 4-wave participant per CU)
int leaf_cus(int64_t m) {
  if (m > reg_max_rows()) return 0;  // the streamed leaf: ordinary launches, no residency
  const int P = leaf_participants(m);
  const int nwv = leaf_waves(m);
  return nwv == 4 ? P : nwv == 2 ? (P + 1) / 2 : (P + 3) / 4;  // a CU holds 4 waves of a full SIMD each
}
// the composed row movement keeps one int per row of the panel in LDS
int64_t compose_max_rows() { return 160 * 1024 / (int64_t)sizeof(int) - 1; }

// Factor the m x LW leaf at A (row/column c0 of the system) in place; leaf =
// the leaf counter of this solve (granule set and tag).
int leaf_factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
                void* ws, int leaf, hipStream_t s, unsigned long long* stamps) {
  if (m < LW || m > max_rows()) return GELIM_FAIL(GELIM_E_ARG, "leaf: m out of range");
  if ((reinterpret_cast<uintptr_t>(A) & 15) || (lda & 1)) return GELIM_FAIL(GELIM_E_ARG, "leaf: alignment");
  if (leaf < 0 || leaf >= (1 << 25)) return GELIM_FAIL(GELIM_E_ARG, "leaf: counter out of range");
  if (leaf_streamed(m))
    return sleaf::factor(A, lda, m, c0, mode, ipiv, pairs, info,
                         static_cast<char*>(ws) + leafk::kKeyBytes + leafk::kRowBytes, s);
  const LeafShape shp = leaf_shape(m);
  leafk::LeafArgs a{};
  a.A = A;
  a.lda = lda;
  a.m = (int)m;
  a.col0 = (int)c0;
  a.P = leaf_participants(m);
  a.leaf = leaf;
  a.ipiv = ipiv;
  a.pairs = pairs;
  a.info = info;
  a.x.key = static_cast<leafk::u32x4*>(ws);
  a.x.row = reinterpret_cast<leafk::u32x4*>(static_cast<char*>(ws) + leafk::kKeyBytes);
  a.stamps = stamps;
  // fused sweep: the key sweep carries every candidate row (P <= 32); the
  // two-hop form (key sweep, then a row load) is what larger P takes inside
  // the leaf (profiles/leaf_fused_vs_2hop.txt)
  constexpr bool fused = true;
  const bool zero = mode != GELIM_PIVOT_PARTIAL;
  if (shp.nwv == 1) {
    if (zero) leafk::launch_leaf_shape<1, 2, 0>(a, fused, s);
    else leafk::launch_leaf_shape<1, 2, 1>(a, fused, s);
  } else if (shp.nwv == 2) {
    if (zero) leafk::launch_leaf_shape<2, 2, 0>(a, fused, s);
    else leafk::launch_leaf_shape<2, 2, 1>(a, fused, s);
  } else {
    if (zero) leafk::launch_leaf_shape<4, 4, 0>(a, fused, s);
    else leafk::launch_leaf_shape<4, 4, 1>(a, fused, s);
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Row movement of a leaf (pairs, may be null) on columns [lbeg, lend) and
// [rbeg, rend) of rows [c0, ...), TRSM of rows [c0, c0 + LW) on the right
// columns below trsm_end.  A: row c0, column 0.  L11 defaults to the leaf
// (row c0, column c0 of A); the distributed solver passes the broadcast
// panel's copy.
int laswp_trsm(double* A, int64_t lda, int64_t c0, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
               int64_t trsm_end, int64_t nrows, const int* pairs, hipStream_t s, const double* L, int64_t ldl) {
  lend = std::max(lend, lbeg);
  rend = std::max(rend, rbeg);
  const int64_t cols = (lend - lbeg) + (rend - rbeg);
  if (cols <= 0) return GELIM_OK;
  if (nrows < LW) return GELIM_FAIL(GELIM_E_ARG, "laswp_trsm: fewer rows than the leaf width");
  if (L == nullptr) {  // L11 is the leaf itself: row c0, column c0 of A
    L = A + c0;
    ldl = lda;
  }
  SwapArgs a{A, lda, (int)c0, (int)lbeg, (int)lend, (int)rbeg, (int)rend, (int)trsm_end, (int)nrows, pairs, L, ldl};
  hipLaunchKernelGGL(laswp_trsm_kernel, dim3((unsigned)((cols + kSwThreads - 1) / kSwThreads)), dim3(kSwThreads), 0,
                     s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Row movement of nleaves consecutive leaves (diagonals c0, c0 + LW, ...;
// pair lists `slot` ints apart) on columns [lbeg, lend) and [rbeg, rend) of
// the n-row system at A (row 0, column 0).
int laswp_panel(double* A, int64_t lda, int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot,
                int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, hipStream_t s, int max_wg) {
  lend = std::max(lend, lbeg);
  rend = std::max(rend, rbeg);
  const int64_t cols = (lend - lbeg) + (rend - rbeg);
  if (cols <= 0 || nleaves <= 0) return GELIM_OK;
  PanelSwapArgs a{A, lda, (int)n, (int)c0, nleaves, pairs, (int)slot, (int)lbeg, (int)lend, (int)rbeg, (int)rend};
  int64_t grid = (cols + 63) / 64;
  if (max_wg > 0) grid = std::min<int64_t>(grid, max_wg);  // <= max_wg CUs (lookahead side stream)
  hipLaunchKernelGGL(laswp_panel_kernel, dim3((unsigned)grid), dim3(64), 0, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Net row movement of nleaves consecutive leaves (diagonals c0, c0 + LW, ...)
// into net (1 + 2 * 64 * nleaves ints, rows relative to c0).
int compose_pairs(int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot, int* net, hipStream_t s) {
  const int64_t m = n - c0;
  if (nleaves <= 0 || m <= 0) return GELIM_OK;
  if (m > compose_max_rows()) return GELIM_FAIL(GELIM_E_ARG, "compose_pairs: too many rows for the LDS row map");
  const size_t lds = sizeof(int) * (size_t)(m + 1);
  static const bool attr = [] {
    return hipFuncSetAttribute((const void*)compose_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(sizeof(int) * (size_t)(compose_max_rows() + 1))) == hipSuccess;
  }();
  if (!attr) return GELIM_FAIL(GELIM_E_HIP, "compose_pairs: LDS attribute refused");
  ComposeArgs a{(int)m, nleaves, pairs, (int)slot, net};
  hipLaunchKernelGGL(compose_kernel, dim3(1), dim3(kCmpThreads), lds, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int laswp_net_max() { return kNsMax; }

// The composed movement on columns [lbeg, lend) and [rbeg, rend) of the rows
// from c0 (A: row c0, column 0); at most laswp_net_max() moved rows.
int laswp_net(double* A, int64_t lda, const int* net, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
              hipStream_t s, int max_wg) {
  lend = std::max(lend, lbeg);
  rend = std::max(rend, rbeg);
  const int64_t cols = (lend - lbeg) + (rend - rbeg);
  if (cols <= 0) return GELIM_OK;
  NetSwapArgs a{A, lda, net, (int)lbeg, (int)lend, (int)rbeg, (int)rend};
  int64_t grid = (cols + kNsCols - 1) / kNsCols;
  if (max_wg > 0) grid = std::min<int64_t>(grid, max_wg);
  hipLaunchKernelGGL(laswp_net_kernel, dim3((unsigned)grid), dim3(kNsThreads), 0, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// U12 = L11^-1 C for the nb rows of C (ldc) over ncols columns, L11 the unit
// lower nb x nb block at L (ldl); nb <= 256, a multiple of 32.
// the fused TRSM kernel (the per-32-row-block TRSM + GEMM sequence it
// replaced is kept for the distributed apply's long panels)
bool trsm_fused() { return true; }

int panel_trsm(double* C, int64_t ldc, int64_t ncols, int64_t nb, const double* L, int64_t ldl, hipStream_t s,
               int max_wg) {
  if (ncols <= 0) return GELIM_OK;
  if (nb <= 0 || nb > kTrNb || nb % LW) return GELIM_FAIL(GELIM_E_ARG, "panel_trsm: nb must be a multiple of 32 <= 256");
  PanelTrsmArgs a{C, ldc, (int)ncols, (int)nb, L, ldl};
  constexpr size_t lds = sizeof(double) * (size_t)kTrNb * ((kTrCols + 1) + (LW + 2));
  static bool attr = [] {
    return hipFuncSetAttribute((const void*)panel_trsm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)lds) == hipSuccess;
  }();
  (void)attr;
  int64_t grid = (ncols + kTrCols - 1) / kTrCols;
  if (max_wg > 0) grid = std::min<int64_t>(grid, max_wg);  // one workgroup per CU (137 KiB of LDS)
  hipLaunchKernelGGL(panel_trsm_kernel, dim3((unsigned)grid), dim3(kTrThreads), lds, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int tail_gemv(const double* A, int64_t lda, int64_t n, int64_t K, const double* x, double* y, double* bnorm,
              hipStream_t s) {
  if (K <= 0) return GELIM_OK;
  hipLaunchKernelGGL(tail_gemv_kernel, dim3((unsigned)((K + 3) / 4)), dim3(256), 0, s, A, lda, (int)n, (int)K, x, y,
                     bnorm);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int fold_info(int* info, const int* tinfo, int64_t K, hipStream_t s) {
  hipLaunchKernelGGL(fold_info_kernel, dim3(1), dim3(64), 0, s, info, tinfo, (int)K);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace big
}  // namespace gelim

// Test entry points: one leaf (m x 32 at dA, the leaf's diagonal at row /
// column c0 of the system) and one laswp + TRSM over the full row width.
extern "C" int gelim_gpu_leaf_factor(double* dA, int64_t lda, int64_t m, int64_t c0, int pivot, int32_t* dipiv,
                                     int32_t* dpairs, int32_t* dinfo, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  void* ws = nullptr;
  HIP_TRY(hipMallocAsync(&ws, gelim::big::workspace_bytes(), s));
  HIP_TRY(hipMemsetAsync(ws, 0, gelim::big::workspace_bytes(), s));
  const int rc = gelim::big::leaf_factor(dA, lda, m, c0, pivot, dipiv, dpairs, dinfo, ws, 0, s, nullptr);
  HIP_TRY(hipFreeAsync(ws, s));
  return rc;
}

// the same with a caller-owned exchange workspace (workspace_bytes(), zeroed
// before the first leaf) and the leaf counter's granule set
extern "C" int gelim_gpu_leaf_factor_ws(double* dA, int64_t lda, int64_t m, int64_t c0, int pivot, int32_t* dipiv,
                                        int32_t* dpairs, int32_t* dinfo, void* ws, int set, void* stream) {
  return gelim::big::leaf_factor(dA, lda, m, c0, pivot, dipiv, dpairs, dinfo, ws, set, (hipStream_t)stream, nullptr);
}

// Diagnostic: one leaf with phase stamps (stamps: P * 32 * 8 u64).
extern "C" int gelim_debug_leaf_stamps(double* dA, int64_t lda, int64_t m, void* ws, unsigned long long* stamps,
                                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  int *ipiv = nullptr, *pairs = nullptr, *info = nullptr;
  HIP_TRY(hipMallocAsync((void**)&ipiv, 64 * 4, s));
  HIP_TRY(hipMallocAsync((void**)&pairs, 256 * 4, s));
  HIP_TRY(hipMallocAsync((void**)&info, 16, s));
  HIP_TRY(hipMemsetAsync(info, 0, 16, s));
  HIP_TRY(hipMemsetAsync(ws, 0, gelim::big::workspace_bytes(), s));
  const int rc = gelim::big::leaf_factor(dA, lda, m, 0, GELIM_PIVOT_PARTIAL, ipiv, pairs, info, ws, 0, s, stamps);
  HIP_TRY(hipFreeAsync(ipiv, s));
  HIP_TRY(hipFreeAsync(pairs, s));
  HIP_TRY(hipFreeAsync(info, s));
  return rc;
}

// max_wg > 0: a grid of at most max_wg workgroups (the lookahead side stream's cap)
extern "C" int gelim_gpu_laswp_panel(double* dA, int64_t lda, int64_t n, int64_t c0, int nleaves,
                                     const int32_t* dpairs, int64_t slot, int64_t lbeg, int64_t lend, int64_t rbeg,
                                     int64_t rend, int max_wg, void* stream) {
  return gelim::big::laswp_panel(dA, lda, n, c0, nleaves, dpairs, slot, lbeg, lend, rbeg, rend, (hipStream_t)stream,
                                 max_wg);
}

extern "C" int gelim_gpu_panel_trsm(double* dC, int64_t ldc, int64_t ncols, int64_t nb, const double* dL, int64_t ldl,
                                    int max_wg, void* stream) {
  return gelim::big::panel_trsm(dC, ldc, ncols, nb, dL, ldl, (hipStream_t)stream, max_wg);
}

extern "C" int64_t gelim_gpu_leaf_workspace_bytes(void) { return (int64_t)gelim::big::workspace_bytes(); }
extern "C" int gelim_gpu_leaf_participants(int64_t m) { return gelim::big::leaf_participants(m); }
extern "C" int64_t gelim_gpu_leaf_max_rows(void) { return gelim::big::max_rows(); }

extern "C" int gelim_gpu_laswp_trsm(double* dA, int64_t lda, int64_t c0, int64_t lend, int64_t rbeg, int64_t rend,
                                    int64_t trsm_end, int64_t nrows, const int32_t* dpairs, void* stream) {
  return gelim::big::laswp_trsm(dA, lda, c0, 0, lend, rbeg, rend, trsm_end, nrows, dpairs, (hipStream_t)stream, nullptr, 0);
}

// the composed form of the same movement (compose + gather/scatter); net:
// 1 + 2 * 64 * nleaves ints of device scratch
extern "C" int gelim_gpu_laswp_net(double* dA, int64_t lda, int64_t n, int64_t c0, int nleaves, const int32_t* dpairs,
                                   int64_t slot, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, int32_t* dnet,
                                   int max_wg, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if ((int64_t)nleaves * 2 * 32 > gelim::big::laswp_net_max())
    return GELIM_FAIL(GELIM_E_ARG, "laswp_net: more moved rows than one pass holds");
  GELIM_TRY(gelim::big::compose_pairs(n, c0, nleaves, dpairs, slot, dnet, s));
  return gelim::big::laswp_net(dA + c0 * lda, lda, dnet, lbeg, lend, rbeg, rend, s, max_wg);
}

