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
// m x 32 is spread over P = ceil(m / 1024) workgroups (4 rows x 32 columns
// per lane, one wave per SIMD), every column's pivot is an exact global
// arg-max (ties to the lowest row, like the reference's strict '>'), and the
// trailing update of each 256-column outer panel is one fp64 MFMA GEMM with
// K = 256 (dgemm.hip) instead of 128 bandwidth-bound rank-2 sweeps.
//
// Leaf protocol, per column J (MI355X_MICROARCH.md "Valid forms", row 1):
//  1. every workgroup finds its best live row (DPP arg-max per wave, one LDS
//     merge behind one barrier);
//  2. wave 0 publishes that row (16-byte sc1 stores), drains (vmcnt 0), then
//     stores ONE 16-byte sc1 granule {key, row, seq = J+1};
//  3. every wave polls the P granules of this column with sc1 loads (lane p
//     reads workgroup p), picks the global winner and loads its row with sc1
//     loads into a wave-private LDS line (no second barrier);
//  4. multipliers and the rank-1 update of the remaining leaf columns in
//     registers.
// Granules and rows are double-buffered by column parity: a workgroup
// overwrites parity J&1 only at column J+2, after every workgroup has
// published column J+1, i.e. after every workgroup has read column J.
// Rows never move inside the leaf (logical pivoting); every wave replays the
// LAPACK interchange sequence in its lanes (<= 64 displaced rows), which
// gives ipiv, the net (dst, src) row movement for the other columns, and --
// for the zero-pivot rule -- the row currently sitting on the diagonal.  At
// the end every lane writes its rows straight to their final LAPACK
// positions (each final position receives exactly one row).
// Every spin is bounded (200 ms) and reports through info[1].
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <utility>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace big {
namespace {

constexpr int NT = 256;            // leaf workgroup: 4 waves, one per SIMD
constexpr int kWaves = NT / 64;
constexpr int LW = 32;             // leaf width
constexpr int R = 4;               // rows per lane
constexpr int kRowsPerWg = NT * R;
constexpr int kMaxP = 64;          // leaf workgroups (m <= 65536)
constexpr int kAuxSc1 = 16;        // buffer-op aux: sc1
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ unsigned lo32(double x) { return (unsigned)__double_as_longlong(x); }
__device__ __forceinline__ unsigned hi32(double x) { return (unsigned)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// 1/p: v_rcp_f64 + two Newton steps (within an ulp of the IEEE quotient)
__device__ __forceinline__ double recip(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  return fma(r, fma(-p, r, 1.0), r);
}

template <typename T>
__device__ __forceinline__ T opq(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

struct LeafArgs {
  double* A;         // leaf top-left: row c0, column c0 of the system
  int64_t lda;
  int m;             // rows n - c0 (>= LW)
  int col0;          // c0 (absolute column / row of the leaf's diagonal)
  int P;             // workgroups
  int set;           // granule set used by this launch (leaf counter & 1)
  int* ipiv;         // ipiv[c0 + J] = absolute row swapped with row c0 + J
  int* pairs;        // [0] = count, then (dst, src) rows relative to c0
  int* info;         // [0] 1 + first zero-pivot column (kept if set), [1] hand-off error
  u32x4* gran;       // [2 sets][2 parities][kMaxP] {key lo, key hi, row, seq}
  double* rows;      // [2 parities][kMaxP][LW] published candidate rows
};

struct alignas(16) LeafLds {
  double cand[2][kWaves][LW];  // each wave's winning row, parity-buffered
  u32x4 ckey[2][kWaves];       // {key lo, key hi, row, -}
  double prow[kWaves][LW];     // each wave's private copy of the pivot row
  int dest[kRowsPerWg];        // final row of a moved local row (-1: unmoved)
  int abort_flag;
};

// ---- the LAPACK interchange replay, one table per wave -----------------------
// Lane e < cnt holds one displaced row: trow (row index, relative to c0) now
// at position tpos.  Rows not in the table sit at their own index.
struct Table {
  int trow, tpos, cnt;
};

__device__ __forceinline__ int table_pos_of(const Table& tb, int row, int lane) {
  const uint64_t m = __ballot(lane < tb.cnt && tb.trow == row);
  return m ? __builtin_amdgcn_readlane(tb.tpos, __ffsll((long long)m) - 1) : row;
}

__device__ __forceinline__ int table_row_at(const Table& tb, int pos, int lane) {
  const uint64_t m = __ballot(lane < tb.cnt && tb.tpos == pos);
  return m ? __builtin_amdgcn_readlane(tb.trow, __ffsll((long long)m) - 1) : pos;
}

// step J: pivot row pr moves to position J, the row at J moves to pr's spot q
__device__ __forceinline__ int table_swap(Table& tb, int J, int pr, int lane) {
  const uint64_t m1 = __ballot(lane < tb.cnt && tb.trow == pr);
  const int q = m1 ? __builtin_amdgcn_readlane(tb.tpos, __ffsll((long long)m1) - 1) : pr;
  if (q == J) return q;
  const uint64_t m2 = __ballot(lane < tb.cnt && tb.tpos == J);
  const int rj = m2 ? __builtin_amdgcn_readlane(tb.trow, __ffsll((long long)m2) - 1) : J;
  int cnt = tb.cnt;
  const int e1 = m1 ? __ffsll((long long)m1) - 1 : cnt++;
  const int e2 = m2 ? __ffsll((long long)m2) - 1 : cnt++;
  if (lane == e1) {
    tb.trow = pr;
    tb.tpos = J;
  }
  if (lane == e2) {
    tb.trow = rj;
    tb.tpos = q;
  }
  tb.cnt = cnt;
  return q;
}

template <int MODE>
__device__ __forceinline__ uint64_t cand_key(double v, bool is_diag, bool ok) {
  return dev::pivot_ukey_t<MODE>(v, is_diag, ok);
}

// put one register row into LDS (the empty asm keeps the per-slot branches
// from being merged into a dynamically indexed access)
__device__ __forceinline__ void put_row(double* dst, const double (&row)[LW]) {
#pragma unroll
  for (int c = 0; c < LW; c += 2) {
    const double x = row[c], y = row[c + 1];
    asm volatile("" ::"v"(x), "v"(y));
    *reinterpret_cast<double2*>(dst + c) = make_double2(x, y);
  }
}

template <int MODE>
struct Leaf {
  template <int J>
  static __device__ __forceinline__ bool col(double (&a)[R][LW], bool (&live)[R], LeafLds& sh, Table& tb,
                                             const LeafArgs& g, int t, int lane, int wave, int base) {
    constexpr int par = J & 1;
    t = opq(t);
    lane = opq(lane);
    // 1. this lane's candidate: best live row (rows grow with the slot, so a
    //    strict '>' keeps the lowest row on ties)
    const int diag = MODE == 0 ? table_row_at(tb, J, lane) : -1;
    uint64_t bk = 0;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int r = base + t + NT * i;
      const uint64_t k = cand_key<MODE>(a[i][J], r == diag, live[i]);
      const bool c = k > bk;
      bk = c ? k : bk;
      bi = c ? i : bi;
    }
    const unsigned brow = (unsigned)(base + t + NT * bi);
    // 2. wave arg-max; the wave's winner parks its row in LDS
    const uint64_t wk = dev::wave_max_u64(bk);
    unsigned wrow = 0xffffffffu;
    if (wk != 0) {
      const uint64_t hold = __ballot(bk == wk);
      int wl;
      if (__popcll(hold) == 1) {
        wl = __ffsll((long long)hold) - 1;
      } else {
        const unsigned mr = dev::wave_min_u32(bk == wk ? brow : 0xffffffffu);
        wl = __ffsll((long long)__ballot(bk == wk && brow == mr)) - 1;
      }
      wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, wl);
      const int wbi = __builtin_amdgcn_readlane(bi, wl);
      if (lane == wl) {
#pragma unroll
        for (int i = 0; i < R; ++i)
          if (wbi == i) put_row(&sh.cand[par][wave][0], a[i]);
      }
    }
    if (lane == 0) sh.ckey[par][wave] = u32x4{(unsigned)wk, (unsigned)(wk >> 32), wrow, 0u};
    __syncthreads();

    // 3. workgroup candidate (wave 0 publishes it) and the global exchange
    {
      const u32x4 kk = sh.ckey[par][lane & (kWaves - 1)];
      const uint64_t key = ((uint64_t)kk.y << 32) | kk.x;
      const bool in = lane < kWaves;
      const uint64_t gk = dev::wave_max_u64(in ? key : 0);
      const unsigned gr = dev::wave_min_u32(in && key == gk ? kk.z : 0xffffffffu);
      const int q = __ffsll((long long)__ballot(in && key == gk && kk.z == gr)) - 1;
      if (wave == 0) {
        const __amdgpu_buffer_rsrc_t rr = rsrc(g.rows + ((int64_t)par * kMaxP + blockIdx.x) * LW, LW * 8);
        if (lane < LW / 2) {
          const double2 v = *reinterpret_cast<const double2*>(&sh.cand[par][q][2 * lane]);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo32(v.x), hi32(v.x), lo32(v.y), hi32(v.y)}, rr, lane * 16, 0,
                                                 kAuxSc1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          const __amdgpu_buffer_rsrc_t rg = rsrc(g.gran + ((g.set * 2 + par) * kMaxP + blockIdx.x), 16);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)gk, (unsigned)(gk >> 32), gr, (unsigned)(J + 1)}, rg, 0,
                                                 0, kAuxSc1);
        }
      }
    }
    // every wave polls the P granules of column J (lane p <-> workgroup p)
    const __amdgpu_buffer_rsrc_t rg = rsrc(g.gran + (g.set * 2 + par) * kMaxP, kMaxP * 16);
    const int pl = lane < g.P ? lane : 0;
    u32x4 gv = __builtin_amdgcn_raw_buffer_load_b128(rg, pl * 16, 0, kAuxSc1);
    if (__ballot(lane < g.P && gv.w != (unsigned)(J + 1)) != 0) {
      const unsigned long long t0 = rtc();
      for (;;) {
        gv = __builtin_amdgcn_raw_buffer_load_b128(rg, pl * 16, 0, kAuxSc1);
        if (__ballot(lane < g.P && gv.w != (unsigned)(J + 1)) == 0) break;
        if (__hip_atomic_load(g.info + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
        if (rtc() - t0 > kSpinTicks) {
          __hip_atomic_store(g.info + 1, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return false;
        }
      }
    }
    // global winner: largest key, lowest row
    const uint64_t key = lane < g.P ? (((uint64_t)gv.y << 32) | gv.x) : 0;
    const uint64_t gk = dev::wave_max_u64(key);
    const unsigned pr = dev::wave_min_u32(lane < g.P && key == gk ? gv.z : 0xffffffffu);
    const int pw = __ffsll((long long)__ballot(lane < g.P && key == gk && gv.z == pr)) - 1;
    // pivot row -> this wave's private LDS line
    {
      const __amdgpu_buffer_rsrc_t rr = rsrc(g.rows + ((int64_t)par * kMaxP + pw) * LW, LW * 8);
      if (lane < LW / 2) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rr, lane * 16, 0, kAuxSc1);
        *reinterpret_cast<double2*>(&sh.prow[wave][2 * lane]) = make_double2(mkd(v.x, v.y), mkd(v.z, v.w));
      }
    }
    // interchange replay (identical in every wave); wave 0 of workgroup 0
    // records the LAPACK pivot
    const int qpos = table_swap(tb, J, (int)pr, lane);
    if (blockIdx.x == 0 && wave == 0 && lane == 0) g.ipiv[g.col0 + J] = g.col0 + qpos;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own LDS line written (wave-local)

    // 4. multipliers and the rank-1 update of columns J+1.. (next column first)
    const double* u = &sh.prow[wave][0];
    const double pv = u[J];
    const bool zero = !(pv != 0.0);
    const double rinv = zero ? 0.0 : recip(pv);
    if (zero && blockIdx.x == 0 && t == 0 && g.info[0] == 0) atomicCAS(g.info, 0, g.col0 + J + 1);
    double l[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      live[i] = live[i] && (base + t + NT * i != (int)pr);
      l[i] = live[i] ? a[i][J] * rinv : 0.0;
      a[i][J] = live[i] ? l[i] : a[i][J];
    }
#pragma unroll
    for (int c = J + 1; c < LW; ++c) {
      const double uc = u[c];
#pragma unroll
      for (int i = 0; i < R; ++i) a[i][c] = fma(-l[i], uc, a[i][c]);
    }
    return true;
  }

  template <int... J>
  static __device__ __forceinline__ bool factor(double (&a)[R][LW], bool (&live)[R], LeafLds& sh, Table& tb,
                                                const LeafArgs& g, int t, int lane, int wave, int base,
                                                std::integer_sequence<int, J...>) {
    return (col<J>(a, live, sh, tb, g, t, lane, wave, base) && ...);
  }
};

template <int MODE>
__global__ __launch_bounds__(NT, 1) void leaf_kernel(LeafArgs g) {
  __shared__ LeafLds sh;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int base = blockIdx.x * kRowsPerWg;
  double a[R][LW];
  bool live[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = base + t + NT * i;
    live[i] = r < g.m;
    const double2* src = reinterpret_cast<const double2*>(g.A + (int64_t)min(r, g.m - 1) * g.lda);
#pragma unroll
    for (int c = 0; c < LW; c += 2) {
      const double2 v = src[c / 2];
      a[i][c] = v.x;
      a[i][c + 1] = v.y;
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) sh.dest[t + NT * i] = -1;
  Table tb{0, 0, 0};
  if (!Leaf<MODE>::factor(a, live, sh, tb, g, t, lane, wave, base, std::make_integer_sequence<int, LW>{}))
    return;

  // net row movement: wave 0 of workgroup 0 publishes it; every workgroup
  // maps its own moved rows to their final positions
  if (wave == 0) {
    if (blockIdx.x == 0) {
      if (lane < tb.cnt) {
        g.pairs[1 + 2 * lane] = tb.tpos;
        g.pairs[2 + 2 * lane] = tb.trow;
      }
      if (lane == 0) g.pairs[0] = tb.cnt;
    }
    if (lane < tb.cnt && tb.trow >= base && tb.trow < base + kRowsPerWg) sh.dest[tb.trow - base] = tb.tpos;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = base + t + NT * i;
    if (r < g.m) {
      const int d = sh.dest[t + NT * i];
      double2* dst = reinterpret_cast<double2*>(g.A + (int64_t)(d < 0 ? r : d) * g.lda);
#pragma unroll
      for (int c = 0; c < LW; c += 2) dst[c / 2] = make_double2(a[i][c], a[i][c + 1]);
    }
  }
  // clear the other granule set for the next leaf launch (this launch's
  // predecessor used it and has finished)
  if (blockIdx.x == 0 && t < 2 * kMaxP) g.gran[((g.set ^ 1) * 2) * kMaxP + t] = u32x4{0u, 0u, 0u, 0u};
}

// ---- row interchanges for the other columns + TRSM of a leaf's U rows -----
// One thread per column of [0, lend) (interchanges only: the L part left of
// the leaf) and of [rbeg, rend) (interchanges, then -- for columns below
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
constexpr int kSwThreads = 256;

struct SwapArgs {
  double* A;
  int64_t lda;
  int c0, lend, rbeg, rend, trsm_end;
  const int* pairs;
};

__global__ __launch_bounds__(kSwThreads) void laswp_trsm_kernel(SwapArgs g) {
  __shared__ double sL[LW][LW + 1];
  __shared__ double xs[LW][kSwThreads];
  __shared__ int sp[1 + 4 * LW];
  const int t = threadIdx.x;
  const int64_t lda = g.lda;
  for (int e = t; e < LW * LW; e += kSwThreads) {
    const int r = e / LW, c = e % LW;
    sL[r][c] = c < r ? g.A[(int64_t)r * lda + g.c0 + c] : 0.0;
  }
  if (t < 1 + 4 * LW) sp[t] = g.pairs && (t == 0 || t <= 2 * g.pairs[0]) ? g.pairs[t] : 0;
  __syncthreads();
  const int np = sp[0];
  const int nleft = g.lend, nright = g.rend - g.rbeg;
  const int idx = blockIdx.x * kSwThreads + t;
  if (idx >= nleft + nright) return;
  const bool right = idx >= nleft;
  const int c = right ? idx - nleft + g.rbeg : idx;
  double* col = g.A + c;
  double gsrc[2 * LW];
#pragma unroll
  for (int e = 0; e < 2 * LW; ++e) gsrc[e] = e < np ? col[(int64_t)sp[2 + 2 * e] * lda] : 0.0;
  if (!right || c >= g.trsm_end) {
#pragma unroll
    for (int e = 0; e < 2 * LW; ++e)
      if (e < np) col[(int64_t)sp[1 + 2 * e] * lda] = gsrc[e];
    return;
  }
#pragma unroll
  for (int j = 0; j < LW; ++j) xs[j][t] = col[(int64_t)j * lda];
#pragma unroll
  for (int e = 0; e < 2 * LW; ++e) {
    if (e < np) {
      const int d = sp[1 + 2 * e];
      if (d < LW) xs[d][t] = gsrc[e];
      else col[(int64_t)d * lda] = gsrc[e];
    }
  }
  double x[LW];
#pragma unroll
  for (int j = 0; j < LW; ++j) x[j] = xs[j][t];
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    __builtin_amdgcn_sched_barrier(0);
    const double xi = x[i];
    col[(int64_t)i * lda] = xi;
#pragma unroll
    for (int j = i + 1; j < LW; ++j) x[j] = fma(-sL[j][i], xi, x[j]);
  }
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

size_t workspace_bytes() { return (size_t)2 * 2 * kMaxP * 16 + (size_t)2 * kMaxP * LW * 8; }
int leaf_width() { return LW; }
int64_t max_rows() { return (int64_t)kMaxP * kRowsPerWg; }

// Factor the m x LW leaf at A (row/column c0 of the system) in place.
int leaf_factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
                void* ws, int set, hipStream_t s) {
  if (m < LW || m > max_rows()) return GELIM_FAIL(GELIM_E_ARG, "leaf: m out of range");
  if ((reinterpret_cast<uintptr_t>(A) & 15) || (lda & 1)) return GELIM_FAIL(GELIM_E_ARG, "leaf: alignment");
  LeafArgs a{};
  a.A = A;
  a.lda = lda;
  a.m = (int)m;
  a.col0 = (int)c0;
  a.P = (int)((m + kRowsPerWg - 1) / kRowsPerWg);
  a.set = set & 1;
  a.ipiv = ipiv;
  a.pairs = pairs;
  a.info = info;
  a.gran = static_cast<u32x4*>(ws);
  a.rows = reinterpret_cast<double*>(static_cast<char*>(ws) + (size_t)2 * 2 * kMaxP * 16);
  if (mode == GELIM_PIVOT_PARTIAL)
    hipLaunchKernelGGL(leaf_kernel<1>, dim3((unsigned)a.P), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL(leaf_kernel<0>, dim3((unsigned)a.P), dim3(NT), 0, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// Row movement of a leaf (pairs, may be null) on columns [0, lend) and
// [rbeg, rend) of rows [c0, ...), TRSM of rows [c0, c0 + LW) on the right
// columns below trsm_end.  A: row c0, column 0.
int laswp_trsm(double* A, int64_t lda, int64_t c0, int64_t lend, int64_t rbeg, int64_t rend, int64_t trsm_end,
               const int* pairs, hipStream_t s) {
  const int64_t cols = lend + std::max<int64_t>(0, rend - rbeg);
  if (cols <= 0) return GELIM_OK;
  SwapArgs a{A, lda, (int)c0, (int)lend, (int)rbeg, (int)rend, (int)trsm_end, pairs};
  hipLaunchKernelGGL(laswp_trsm_kernel, dim3((unsigned)((cols + kSwThreads - 1) / kSwThreads)), dim3(kSwThreads), 0,
                     s, a);
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
  const int rc = gelim::big::leaf_factor(dA, lda, m, c0, pivot, dipiv, dpairs, dinfo, ws, 0, s);
  HIP_TRY(hipFreeAsync(ws, s));
  return rc;
}

// the same with a caller-owned exchange workspace (workspace_bytes(), zeroed
// before the first leaf) and the leaf counter's granule set
extern "C" int gelim_gpu_leaf_factor_ws(double* dA, int64_t lda, int64_t m, int64_t c0, int pivot, int32_t* dipiv,
                                        int32_t* dpairs, int32_t* dinfo, void* ws, int set, void* stream) {
  return gelim::big::leaf_factor(dA, lda, m, c0, pivot, dipiv, dpairs, dinfo, ws, set, (hipStream_t)stream);
}

extern "C" int64_t gelim_gpu_leaf_workspace_bytes(void) { return (int64_t)gelim::big::workspace_bytes(); }

extern "C" int gelim_gpu_laswp_trsm(double* dA, int64_t lda, int64_t c0, int64_t lend, int64_t rbeg, int64_t rend,
                                    int64_t trsm_end, const int32_t* dpairs, void* stream) {
  return gelim::big::laswp_trsm(dA, lda, c0, lend, rbeg, rend, trsm_end, dpairs, (hipStream_t)stream);
}
