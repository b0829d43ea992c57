// Panel factorisation for the blocked LU — the latency-critical part of
// Gaussian elimination on MI355X.
//
// What it computes: the reference's pivot search + row swap + elimination
// (getPivot / computeGauss, OpenMP_and_MPI/gauss_openmp/gauss_external_input.c
// :123-182) restricted to a tall m x w column panel, LAPACK-getf2 style:
// for j in 0..w-1 choose the pivot row p (PARTIAL: argmax |a|, ties to the
// lowest row like the reference's strict '>'; ZERO: the reference's internal
// rule), L[r][j] = a[r][j] / a[p][j], rank-1 update of the remaining panel
// columns; on exit rows are in LAPACK order and piv[] holds LAPACK's
// sequential interchanges (local row indices).
//
// How (MI355X-first):
//  * ONE workgroup of NT threads (512 = 2 wave64s per SIMD, so one wave's
//    pivot-search latency hides under the other's FMAs) holds the whole panel
//    in VGPRs: thread t owns rows t, t+NT, ... (R rows x W columns <= 64
//    doubles per lane, no AGPR spills).
//  * rows never move during the column loop ("logical pivoting"): a chosen
//    row is retired through a per-lane bit mask; the interchange sequence and
//    the final row placement are reconstructed once at the end;
//  * one workgroup barrier per column: each wave's arg-max is found with a
//    DPP max-scan of the key's high word + one ballot (the exact 64-bit
//    max / lowest-row tie-break runs only when lanes share the high word);
//    the winning lane writes its row into an LDS slot; after the barrier every
//    wave reduces the per-wave candidates itself and reads the pivot row;
//    slots are double-buffered by column parity, which is what makes one
//    barrier per column race-free;
//  * the panel is read and written once, coalesced, staged through LDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <utility>
#include <vector>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kMaxWaves = 8;

template <int W>
struct alignas(16) PanelLds {
  double cand_row[2][kMaxWaves][W];       // each wave's winning row (parity-buffered)
  uint64_t cand_key[2][kMaxWaves];        // the wave's winning key
  unsigned cand_row_idx[2][kMaxWaves];
  int sel[W];         // physical (original) row chosen at each step
  int pos_of[2 * W];  // compact row id -> compact position
  int row_at[2 * W];  // compact position -> compact row id
  int piv[W];
};

extern __shared__ __attribute__((aligned(16))) char g_panel_dyn_lds[];

// Value barrier: stops LLVM from folding a select over register-array
// elements into a dynamically indexed access (which demotes the array to
// scratch memory).
__device__ __forceinline__ double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// Diagnostic per-step stamps (STAMP builds only), kept in registers.
struct StepStamps {
  unsigned long long v[6];
};

// Exact wave arg-max of (key, row): largest key, lowest row on ties.
__device__ __forceinline__ void wave_argmax_exact(uint64_t best, unsigned brow, uint64_t& wkey,
                                                  unsigned& wrow) {
  wkey = dev::wave_max_u64(best);
  const uint64_t h2 = __ballot(best == wkey);
  if (__popcll(h2) == 1)
    wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, __ffsll((long long)h2) - 1);
  else
    wrow = dev::wave_min_u32(best == wkey ? brow : 0xffffffffu);
}

template <int NT, int R, int W, int MODE, bool STAMP>
struct Panel {
  static constexpr int kWaves = NT / dev::kWave;
  static_assert(kWaves <= kMaxWaves && (kWaves & (kWaves - 1)) == 0, "waves: power of two <= 8");

  template <int J>
  static __device__ __forceinline__ void stamp(StepStamps& ss, int slot) {
    if constexpr (STAMP) {
      if (J == 4) ss.v[slot] = stamp_now();
    }
  }

  // One column step J (compile time, so every register index is static).
  // The VALU instruction count per column is what bounds this loop (every
  // wave executes the whole step; 2 waves share a SIMD at NT = 512), so the
  // step is written to minimise it: per-slot liveness as lane masks, a
  // hi-word DPP arg-max with one ballot, a publish of only columns >= J, and
  // a lane-parallel DPP merge of the per-wave candidates.
  template <int J>
  static __device__ __forceinline__ void step(double (&a)[R][W], bool (&live)[R], int (&retj)[R],
                                              int (&pos)[R], int (&rec)[4], PanelLds<W>& sh, int t, int lane,
                                              int wave,
                                              bool active, int w, int row0,
                                              int* __restrict__ info, StepStamps& ss,
                                              double* __restrict__ Lout, int ldL,
                                              __amdgpu_buffer_rsrc_t lrs) {
    if (J >= w) return;  // uniform across the workgroup
    constexpr int par = J & 1;
    stamp<J>(ss, 0);

    uint64_t wkey = 0;
    unsigned wrow = 0xffffffffu;
    if (active) {  // uniform per wave: the wave holds panel rows
      // 1. local candidate over this lane's live rows; its reciprocal is
      //    computed speculatively (hidden under the DPP ladder) and published
      //    in place of the pivot value, so no division follows the barrier
      uint64_t best = 0;
      unsigned brow = 0xffffffffu;
      double bval = 0.0;
      if constexpr (MODE == 1) {
        // PARTIAL: compare magnitudes as fp64 (one v_cmp per row instead of
        // the 64-bit key arithmetic): max(|a|, 0) ranks NaN like zero, a
        // retired row gets a negative magnitude (hi word only) and never
        // beats the -0.5 start; the integer key bits(m)+1 (0: none) is built
        // once per lane -- the same order as pivot_ukey_t
        double bm = -0.5;
#pragma unroll
        for (int i = 0; i < R; ++i) {
          // one v_max_f64 with the |.| modifier (fmax() would add a
          // canonicalising max per row)
          double mg;
          asm("v_max_f64 %0, |%1|, 0" : "=v"(mg) : "v"(a[i][J]));
          const uint64_t mb = (uint64_t)__double_as_longlong(mg);
          const double m = __longlong_as_double(
              (long long)((live[i] ? (mb >> 32) : 0xbff00000ull) << 32 | (mb & 0xffffffffull)));
          const bool better = m > bm;  // increasing rows: '>' keeps the lowest row on ties
          bm = better ? m : bm;
          brow = better ? (unsigned)(t + i * NT) : brow;
          bval = better ? a[i][J] : bval;
        }
        best = bm >= 0.0 ? (uint64_t)__double_as_longlong(bm) + 1 : 0;
      } else {
        // ZERO rule (Pthreads/Version-1/gauss_internal_input.c:75-121): the
        // row at POSITION J after the earlier interchanges is "the diagonal";
        // rows never move here, so each lane tracks its rows' positions and
        // the key is class<<32 | ~position (class 3 non-zero diagonal, 2 other
        // non-zero, 1 zero): the max key is the reference's choice, and keys
        // are unique, so no row tie-break is ever needed
#pragma unroll
        for (int i = 0; i < R; ++i) {
          const uint64_t cls = dev::pivot_ukey_t<MODE>(a[i][J], pos[i] == J, live[i]);
          const uint64_t key = cls == 0 ? 0 : (cls << 32) | (0xffffffffu - (unsigned)pos[i]);
          const bool better = key > best;
          best = better ? key : best;
          brow = better ? (unsigned)(t + i * NT) : brow;
          bval = better ? a[i][J] : bval;
        }
      }
      // reciprocal of this lane's candidate, computed by every lane BEFORE the
      // ladder (the value barrier stops LLVM from sinking it into the
      // winner's publish branch, onto the critical path): v_rcp_f64 + two
      // Newton steps, within an ulp of the IEEE quotient
      double lrd = 0.0;
      {
        const double r0 = __builtin_amdgcn_rcp(bval);
        const double r1 = fma(r0, fma(-bval, r0, 1.0), r0);
        lrd = (bval != 0.0) ? fma(r1, fma(-bval, r1, 1.0), r1) : 0.0;
        lrd = opaque(lrd);
      }
      // 2. wave arg-max: DPP max of the high word + one ballot; exact path
      //    only for high-word ties (or all-zero / denormal columns)
      if constexpr (MODE == 1) {
        const unsigned bhi = (unsigned)(best >> 32);
        const unsigned hmax = dev::wave_max_u32(bhi);
        const uint64_t holders = __ballot(bhi == hmax);
        if (hmax != 0 && __popcll(holders) == 1) {
          const int wl = __ffsll((long long)holders) - 1;
          wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, wl);
          wkey = ((uint64_t)hmax << 32) | (unsigned)__builtin_amdgcn_readlane((int)(unsigned)best, wl);
        } else {
          wave_argmax_exact(best, brow, wkey, wrow);
        }
      } else {
        wave_argmax_exact(best, brow, wkey, wrow);
      }
      stamp<J>(ss, 1);
      // the lane holding the wave's winner publishes columns >= J of its row
      // (column J carries the reciprocal of the pivot)
      if (wkey != 0 && (int)(wrow & (NT - 1)) == t) {
        const int ip = (int)(wrow / NT);
#pragma unroll
        for (int i = 0; i < R; ++i)
          if (i == ip) {
#pragma unroll
            for (int c = J & ~1; c < W; c += 2) {
              // input-only value barrier: keeps one store branch per slot
              // (a merged select would index a[] dynamically -> scratch)
              const double x0 = (c == J) ? lrd : a[i][c];
              const double x1 = (c + 1 == J) ? lrd : a[i][c + 1];
              asm volatile("" ::"v"(x0), "v"(x1));
              *reinterpret_cast<double2*>(&sh.cand_row[par][wave][c]) = make_double2(x0, x1);
            }
          }
      }
    }
    if (lane == 0) {
      sh.cand_key[par][wave] = wkey;
      sh.cand_row_idx[par][wave] = wrow;
    }
    stamp<J>(ss, 2);
    __syncthreads();
    stamp<J>(ss, 3);

    // 3. one LDS round trip: lane q < kWaves reads wave q's key, and every
    //    lane reads a slice of all candidate rows (LPR lanes per row, DPL
    //    doubles per lane) — the winner's values are then broadcast with
    //    v_readlane into SGPRs instead of every wave re-reading the row
    constexpr int DPL = (W * kWaves >= 128) ? 2 : 1;
    constexpr int LPR = W / DPL;
    uint64_t k = sh.cand_key[par][lane & (kWaves - 1)];
    unsigned r = sh.cand_row_idx[par][lane & (kWaves - 1)];
    double cv[DPL];
    {
      const int q = lane / LPR, c0 = (lane % LPR) * DPL;
      const int qq = q < kWaves ? q : 0;
      if constexpr (DPL == 2) {
        const double2 v = *reinterpret_cast<const double2*>(&sh.cand_row[par][qq][c0]);
        cv[0] = v.x;
        cv[1] = v.y;
      } else {
        cv[0] = sh.cand_row[par][qq][c0];
      }
    }
    // fast path: a max ladder over the waves' key HIGH words (one DPP max per
    // level) + one ballot; the exact (key, lowest row) ladder only when two
    // waves share the high word (or no wave has a candidate)
    uint64_t gkey;
    unsigned p;
    {
      const unsigned khi = (unsigned)(k >> 32);
      unsigned hm = khi;
#pragma unroll
      for (int sft = 1; sft < kWaves; sft <<= 1) {
        if (sft == 1) hm = max(hm, dev::dpp_u32<dev::kDppRowShr1, 0xf, 0xf>(0u, hm));
        else if (sft == 2) hm = max(hm, dev::dpp_u32<dev::kDppRowShr2, 0xf, 0xf>(0u, hm));
        else hm = max(hm, dev::dpp_u32<dev::kDppRowShr4, 0xf, 0xf>(0u, hm));
      }
      const unsigned hmax = (unsigned)__builtin_amdgcn_readlane((int)hm, kWaves - 1);
      const uint64_t holders = __ballot(khi == hmax) & ((1ull << kWaves) - 1ull);
      if (hmax != 0 && __popcll(holders) == 1) {
        const int wl = __ffsll((long long)holders) - 1;
        gkey = ((uint64_t)hmax << 32) | (unsigned)__builtin_amdgcn_readlane((int)(unsigned)k, wl);
        p = (unsigned)__builtin_amdgcn_readlane((int)r, wl);
      } else {
#pragma unroll
        for (int sft = 1; sft < kWaves; sft <<= 1) {
          unsigned khi2 = (unsigned)(k >> 32), klo = (unsigned)k, k2hi, k2lo, r2;
          if (sft == 1) {
            k2hi = dev::dpp_u32<dev::kDppRowShr1, 0xf, 0xf>(0u, khi2);
            k2lo = dev::dpp_u32<dev::kDppRowShr1, 0xf, 0xf>(0u, klo);
            r2 = dev::dpp_u32<dev::kDppRowShr1, 0xf, 0xf>(0xffffffffu, r);
          } else if (sft == 2) {
            k2hi = dev::dpp_u32<dev::kDppRowShr2, 0xf, 0xf>(0u, khi2);
            k2lo = dev::dpp_u32<dev::kDppRowShr2, 0xf, 0xf>(0u, klo);
            r2 = dev::dpp_u32<dev::kDppRowShr2, 0xf, 0xf>(0xffffffffu, r);
          } else {
            k2hi = dev::dpp_u32<dev::kDppRowShr4, 0xf, 0xf>(0u, khi2);
            k2lo = dev::dpp_u32<dev::kDppRowShr4, 0xf, 0xf>(0u, klo);
            r2 = dev::dpp_u32<dev::kDppRowShr4, 0xf, 0xf>(0xffffffffu, r);
          }
          const uint64_t k2 = ((uint64_t)k2hi << 32) | k2lo;
          const bool better = k2 > k || (k2 == k && r2 < r);
          k = better ? k2 : k;
          r = better ? r2 : r;
        }
        gkey = ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(k >> 32), kWaves - 1) << 32) |
               (unsigned)__builtin_amdgcn_readlane((int)(unsigned)k, kWaves - 1);
        p = (unsigned)__builtin_amdgcn_readlane((int)r, kWaves - 1);
      }
    }
    const int pw = (int)((p & (NT - 1)) >> 6);  // wave that published the pivot row
    auto bcast = [&](int c) -> double {         // u[c] of the pivot row (uniform)
      const int src = pw * LPR + c / DPL;
      const uint64_t bits = (uint64_t)__double_as_longlong(cv[c % DPL]);
      const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(bits >> 32), src);
      const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)bits, src);
      return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    };
    const double rd = bcast(J);
    double uc[W];
    // the critical operand (column J+1, whose update feeds the next pivot
    // search) by v_readlane; the rest of the pivot row as uniform-address
    // LDS reads (broadcast, 2 doubles per ds_read_b128 instead of 4 VALU
    // readlanes), consumed after column J+1 is done
    if constexpr (J + 1 < W) uc[J + 1] = bcast(J + 1);
    {
      const double* prow = sh.cand_row[par][pw];
      constexpr int c0 = (J + 2) & ~1;
#pragma unroll
      for (int c = c0; c < W; c += 2) {
        const double2 v = *reinterpret_cast<const double2*>(prow + c);
        if (c >= J + 2) uc[c] = v.x;
        if (c + 1 >= J + 2) uc[c + 1] = v.y;
      }
    }
    if (t == 0) {
      sh.sel[J] = (int)p;
      const bool zpiv = MODE == 1 ? gkey <= 1 : (gkey >> 32) <= 1;
      if (zpiv && info && *info == 0) *info = row0 + J + 1;  // zero pivot
    }
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool won = t + i * NT == (int)p;
      retj[i] = won ? J : retj[i];  // the step this row was chosen at (dest, below)
      live[i] = live[i] && !won;
    }
    if constexpr (MODE == 0) {
      // interchange of positions J and pos(p) (p's position is in its key)
      const int posp = gkey != 0 ? (int)(0xffffffffu - (unsigned)gkey) : J;
#pragma unroll
      for (int i = 0; i < R; ++i)
        pos[i] = (t + i * NT == (int)p) ? J : (pos[i] == J ? posp : pos[i]);
    }
    stamp<J>(ss, 4);

    // 4. multipliers + rank-1 update of every live row (retired rows: l = 0);
    //    column J+1 first — the next step's pivot search depends only on it
    if (active) {
      double l[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        l[i] = live[i] ? a[i][J] * rd : 0.0;
        a[i][J] = live[i] ? l[i] : a[i][J];
      }
      if constexpr (J + 1 < W) {
#pragma unroll
        for (int i = 0; i < R; ++i) a[i][J + 1] = fma(-l[i], uc[J + 1], a[i][J + 1]);
      }
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = J + 2; c < W; ++c) a[i][c] = fma(-l[i], uc[c], a[i][c]);
    }
    if constexpr (STAMP) {
      if (J == 4) {
        asm volatile("" ::"v"(a[R - 1][W - 1]));
        ss.v[5] = stamp_now();
      }
    }
    // 5. column J is final for every row now (multipliers of the live rows,
    //    U entries of the retired ones): store it column-major in physical
    //    row order while the next columns are factored — coalesced, and off
    //    the critical path.  Rows >= m land in the buffer's padding
    //    (ldL >= NT * R); the <= 2w moved rows are fixed up at the end.
    if (Lout != nullptr) {
#pragma unroll
      for (int i = 0; i < R; ++i)
        dev::store_buf_wt(lrs, (uint32_t)t * 8u, (uint32_t)(J * ldL + i * NT) * 8u, a[i][J]);
    }
    // 6. wave 0: step J of the LAPACK interchange replay (compact ids: rows
    //    < w keep their index, the row chosen at step j >= w is w + j; lane x
    //    holds pos_of[x] (rec[0]), row_at[x] (rec[1]), sel[x] (rec[2]) and
    //    the LAPACK ipiv (rec[3])) -- done column by column here instead of
    //    as a 16-step serial chain after the loop
    if (wave == 0) {
      rec[2] = (lane == J) ? (int)p : rec[2];  // sel[J] (read below when p is new)
      const int idp = (int)p < w ? (int)p : w + J;
      const int cur = __builtin_amdgcn_readlane(rec[0], idp);
      const int other = __builtin_amdgcn_readlane(rec[1], J);
      rec[1] = (lane == J) ? idp : rec[1];  // row_at[J] = idp; row_at[cur] = other
      rec[1] = (lane == cur) ? other : rec[1];
      rec[0] = (lane == idp) ? J : rec[0];  // pos_of[idp] = J; pos_of[other] = cur
      rec[0] = (lane == other) ? cur : rec[0];
      if (Lout == nullptr) {  // standalone panel: LAPACK ipiv
        const int pj = cur < w ? cur : __builtin_amdgcn_readlane(rec[2], cur < w ? 0 : cur - w);
        rec[3] = (lane == J) ? pj : rec[3];
      }
    }
  }

  template <int... J>
  static __device__ __forceinline__ void steps(double (&a)[R][W], bool (&live)[R], int (&retj)[R],
                                               int (&pos)[R], int (&rec)[4], PanelLds<W>& sh, int t, int lane,
                                               int wave,
                                               bool active, int w, int row0, int* info,
                                               StepStamps& ss, double* Lout, int ldL,
                                               __amdgpu_buffer_rsrc_t lrs,
                                               std::integer_sequence<int, J...>) {
    (step<J>(a, live, retj, pos, rec, sh, t, lane, wave, active, w, row0, info, ss, Lout, ldL, lrs), ...);
  }

  // LDS staging tile: NT rows x W doubles in 16-byte chunks, XOR-swizzled by
  // row so per-row ds_read_b128 / ds_write_b128 spread over the banks.
  static __device__ __forceinline__ int swz(int row, int ch) { return ch ^ (row & (W / 2 - 1)); }

  static __device__ __forceinline__ void stage_in(double (&a)[R][W], const double* __restrict__ P,
                                                  int64_t ldp, int m, int t) {
    constexpr int CH = W / 2;     // 16-byte chunks per row
    constexpr int RPP = NT / CH;  // rows per coalesced pass
    double2* tile = reinterpret_cast<double2*>(g_panel_dyn_lds);
    const int ch = t % CH;
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int pass = 0; pass < CH; ++pass) {
        const int rl = pass * RPP + t / CH;
        const int lr = i * NT + rl;
        double2 v = make_double2(0.0, 0.0);
        if (lr < m) v = *reinterpret_cast<const double2*>(P + (int64_t)lr * ldp + 2 * ch);
        tile[rl * CH + swz(rl, ch)] = v;
      }
      __syncthreads();
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const double2 v = tile[t * CH + swz(t, c)];
        a[i][2 * c] = v.x;
        a[i][2 * c + 1] = v.y;
      }
      __syncthreads();
    }
  }

  // Coalesced loads of EVERY slot issued up front (one memory latency, 8
  // cache lines per instruction instead of 64), then a swizzled LDS transpose
  // slot by slot into the row-per-thread layout.  Rows >= m read row m-1.
  static __device__ __forceinline__ void stage_in_all(double (&a)[R][W], const double* __restrict__ P,
                                                      int64_t ldp, int m, int t) {
    constexpr int CH = W / 2;     // 16-byte chunks per row
    constexpr int RPP = NT / CH;  // rows per coalesced pass
    double2* tile = reinterpret_cast<double2*>(g_panel_dyn_lds);
    const int ch = t % CH;
    // a[i] first holds slot i's coalesced chunks (chunk `ch` of rows
    // pass*RPP + t/CH), then, after the transpose, this thread's row
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int pass = 0; pass < CH; ++pass) {
        const int lr = min(i * NT + pass * RPP + t / CH, m - 1);
        const double2 v = *reinterpret_cast<const double2*>(P + (int64_t)lr * ldp + 2 * ch);
        a[i][2 * pass] = v.x;
        a[i][2 * pass + 1] = v.y;
      }
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int pass = 0; pass < CH; ++pass) {
        const int rl = pass * RPP + t / CH;
        tile[rl * CH + swz(rl, ch)] = make_double2(a[i][2 * pass], a[i][2 * pass + 1]);
      }
      __syncthreads();
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        const double2 v = tile[t * CH + swz(t, c)];
        a[i][2 * c] = v.x;
        a[i][2 * c + 1] = v.y;
      }
      __syncthreads();
    }
  }

  static __device__ __forceinline__ void stage_out(const double (&a)[R][W], const int (&dest)[R],
                                                   double* __restrict__ P, int64_t ldp, int m,
                                                   int t) {
    constexpr int CH = W / 2;
    constexpr int RPP = NT / CH;
    double2* tile = reinterpret_cast<double2*>(g_panel_dyn_lds);
    int* dst_row = reinterpret_cast<int*>(g_panel_dyn_lds + sizeof(double2) * NT * CH);
    const int ch = t % CH;
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
      for (int c = 0; c < CH; ++c)
        tile[t * CH + swz(t, c)] = make_double2(a[i][2 * c], a[i][2 * c + 1]);
      dst_row[t] = dest[i];
      __syncthreads();
#pragma unroll
      for (int pass = 0; pass < CH; ++pass) {
        const int rl = pass * RPP + t / CH;
        const int lr = i * NT + rl;
        if (lr < m)
          *reinterpret_cast<double2*>(P + (int64_t)dst_row[rl] * ldp + 2 * ch) =
              tile[rl * CH + swz(rl, ch)];
      }
      __syncthreads();
    }
  }

  static constexpr size_t stage_bytes() { return sizeof(double) * NT * W + sizeof(int) * NT; }

  // Direct register IO: every lane moves its own rows with 16-byte accesses;
  // all R*W/2 requests are in flight at once (one memory latency instead of
  // R staged passes), at the cost of uncoalesced per-instruction addresses.
  static __device__ __forceinline__ void load_direct(double (&a)[R][W], const double* __restrict__ P,
                                                     int64_t ldp, int m, int t) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      // rows >= m read row m-1 (never live, values unused): no branch, so
      // every load of the strip is in flight at once
      const int lr = min(t + i * NT, m - 1);
      const double2* src = reinterpret_cast<const double2*>(P + (int64_t)lr * ldp);
#pragma unroll
      for (int c = 0; c < W / 2; ++c) {
        const double2 v = src[c];
        a[i][2 * c] = v.x;
        a[i][2 * c + 1] = v.y;
      }
    }
  }

  // Column-major source (the narrow kernel's strip buffer): every load of the
  // panel in flight at once, column 0 first — coalesced 8-byte loads (lanes =
  // consecutive rows), no LDS transpose, and the compiler's per-register
  // vmcnt waits let column 0's pivot search start before the later columns
  // have arrived.
  static __device__ __forceinline__ void load_colmajor(double (&a)[R][W], const double* __restrict__ Pin,
                                                       int64_t ld, int m, int w, int t) {
#pragma unroll
    for (int c = 0; c < W; ++c)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double v = Pin[(int64_t)c * ld + min(t + i * NT, m - 1)];
        a[i][c] = c < w ? v : 0.0;
      }
  }

  static __device__ __forceinline__ void store_direct(const double (&a)[R][W], const int (&dest)[R],
                                                      double* __restrict__ P, int64_t ldp, int m,
                                                      int t) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      if (lr < m) {
        double2* dst = reinterpret_cast<double2*>(P + (int64_t)dest[i] * ldp);
#pragma unroll
        for (int c = 0; c < W / 2; ++c) dst[c] = make_double2(a[i][2 * c], a[i][2 * c + 1]);
      }
    }
  }
};

template <int NT, int R, int W, int MODE, bool STAMP>
__device__ __forceinline__ void panel_body(double* __restrict__ P, int64_t ldp, int m, int w,
                                           int row0, int* __restrict__ piv,
                                           int* __restrict__ info,
                                           unsigned long long* __restrict__ stamps,
                                           int* __restrict__ pairs, PanelLds<W>& sh,
                                           int io = 0, const double* Pin = nullptr,
                                           int64_t ldin = 0, double* __restrict__ Lout = nullptr,
                                           int ldL = 0, bool pin_colmajor = false) {
  // the panel is read from Pin (default: P itself) and written to P; with
  // Lout, the factored panel goes column-major (ld ldL, final row order) to
  // Lout and only the U11 rows to P (the fused step schedule)
  if (Pin == nullptr) {
    Pin = P;
    ldin = ldp;
  }
  using K = Panel<NT, R, W, MODE, STAMP>;
  const int t = threadIdx.x;
  const int lane = t & (dev::kWave - 1);
  const int wave = t >> 6;
  unsigned long long t0 = 0;
  if constexpr (STAMP) t0 = stamp_now();

  double a[R][W];
  // full-width panels with 16-byte aligned rows are staged through LDS so the
  // global loads are coalesced (W/2 lanes per row segment)
  const bool staged = (w == W) && (W % 2 == 0) && ((((uintptr_t)P) & 15) == 0) && (ldp % 2 == 0) &&
                      ((((uintptr_t)Pin) & 15) == 0) && (ldin % 2 == 0);
  if (pin_colmajor) {
    K::load_colmajor(a, Pin, ldin, m, w, t);
  } else if (staged && io == 1) {
    K::load_direct(a, Pin, ldin, m, t);
  } else if (staged && io == 2) {
    K::stage_in_all(a, Pin, ldin, m, t);
  } else if (staged) {
    K::stage_in(a, Pin, ldin, m, t);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      const double* src = Pin + (int64_t)min(lr, m - 1) * ldin;  // clamped: no divergent loads
#pragma unroll
      for (int c = 0; c < W; ++c) {
        const double v = src[min(c, w - 1)];
        a[i][c] = (lr < m && c < w) ? v : 0.0;
      }
    }
  }
  bool live[R];
  int retj[R];
  int pos[R];  // ZERO rule: current position of each row (unused for PARTIAL)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    live[i] = t + i * NT < m;
    retj[i] = 0;
    pos[i] = t + i * NT;
  }
  const __amdgpu_buffer_rsrc_t lrs = dev::buffer_rsrc(Lout, (uint64_t)W * (uint64_t)ldL * 8);
  const bool active = wave * dev::kWave < m;  // the wave holds panel rows
  unsigned long long t1 = 0;
  if constexpr (STAMP) {
    __syncthreads();
    t1 = stamp_now();
  }

  StepStamps ss{};
  int rec[4] = {lane, lane, 0, 0};  // wave 0: interchange replay state (see step 6)
  K::steps(a, live, retj, pos, rec, sh, t, lane, wave, active, w, row0, info, ss, Lout, ldL, lrs,
           std::make_integer_sequence<int, W>{});
  unsigned long long t2 = 0;
  if constexpr (STAMP) t2 = stamp_now();

  // Reconstruct LAPACK's sequential interchanges from the selection order.
  // Compact ids: rows < w keep their index; a chosen row >= w selected at
  // step j gets id w + j.  Compact positions use the same numbering (the
  // only positions >= w ever touched are original places of chosen rows).
  // Wave 0 runs the w-step simulation in registers (lane x holds pos_of[x]
  // and row_at[x]; every index is wave-uniform, so reads are v_readlane and
  // writes are lane selects) — no serial LDS round trips.
  if (wave == 0) {
    // the replay ran column by column (step 6): rec = pos_of, row_at, sel, ipiv
    const int selv = rec[2];
    const int pos = rec[0], rat = rec[1], pivv = rec[3];
    if (lane < w) sh.piv[lane] = pivv;
    if (lane < 2 * w) {
      sh.pos_of[lane] = pos;
      sh.row_at[lane] = rat;
    }
    // net row movement as (dst, src) pairs for the trailing-column kernels:
    // new_row[dst] = old_row[src] over the <= 2w touched rows
    if (pairs) {
      // compact position w+j stands for actual position sel[j] only when
      // that row lies below the panel top (otherwise it is unused)
      const int xs = (lane >= w && lane < 2 * w) ? lane - w : 0;
      const int selx = __shfl(selv, xs);
      const int id = rat;
      const int selid = __shfl(selv, (id >= w && id < 2 * w) ? id - w : 0);
      const int ap = lane < w ? lane : selx;
      const int ar = id < w ? id : selid;
      const bool emit = lane < 2 * w && !(lane >= w && selx < w) && ap != ar;
      const uint64_t mask = __ballot(emit);
      const int k = __popcll(mask & ((1ull << lane) - 1ull));
      // agent-scope (sc1) stores: the fused narrow update reads them in the
      // same launch, possibly from another XCD
      if (emit) {
        __hip_atomic_store(pairs + 1 + 2 * k, ap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(pairs + 2 + 2 * k, ar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) __hip_atomic_store(pairs, (int)__popcll(mask), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  unsigned long long tr = 0;
  if constexpr (STAMP) tr = stamp_now();
  unsigned long long ta = 0, tb = 0, tc = 0;
  if constexpr (STAMP) ta = stamp_now();
  __syncthreads();  // the replay's pos_of / sel are in LDS
  if constexpr (STAMP) tb = stamp_now();

  // final position of every physical row
  int dest[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * NT;
    int d = lr;
    int id = -1;
    if (lr < w) {
      id = lr;
    } else if (lr < m && !live[i]) {
      id = w + retj[i];
    }
    if (id >= 0) {
      const int cp = sh.pos_of[id];
      d = cp < w ? cp : sh.sel[cp - w];
    }
    dest[i] = d;
  }
  if constexpr (STAMP) tc = stamp_now();
  if (Lout != nullptr) {
    // every lane's early column stores complete before any fix-up store to
    // the same rows (another lane's): drained only now, so the destination
    // computation above ran while the last columns' stores were in flight
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // rows that moved overwrite their final position's early store; the
    // rows landing in the top w (U11) also go to P for the back substitution
    const __amdgpu_buffer_rsrc_t urs = dev::buffer_rsrc(P, (uint64_t)W * (uint64_t)ldp * 8);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      if (lr < m && dest[i] != lr) {
#pragma unroll
        for (int c = 0; c < W; ++c)
          if (c < w) dev::store_buf_wt(lrs, (uint32_t)dest[i] * 8u, (uint32_t)(c * ldL) * 8u, a[i][c]);
      }
      if (lr < m && dest[i] < w) {
        const uint32_t ro = (uint32_t)((int64_t)dest[i] * ldp * 8);
#pragma unroll
        for (int c = 0; c < W; ++c)
          if (c < w) dev::store_buf(urs, ro, (uint32_t)c * 8u, a[i][c]);
      }
    }
  } else if (staged && io == 1) {
    K::store_direct(a, dest, P, ldp, m, t);
  } else if (staged) {
    K::stage_out(a, dest, P, ldp, m, t);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      if (lr < m) {
        double* dst = P + (int64_t)dest[i] * ldp;
#pragma unroll
        for (int c = 0; c < W; ++c)
          if (c < w) dst[c] = a[i][c];
      }
    }
  }
  if (t < w) piv[t] = sh.piv[t];
  if constexpr (STAMP) {
    __syncthreads();
    if (t == 0) {
      stamps[0] = t0;
      stamps[1] = t1;
      stamps[2] = t2;
      stamps[3] = stamp_now();
      stamps[4] = ta;
      stamps[5] = tb;
      stamps[6] = tc;
      stamps[7] = tr;
      for (int k = 0; k < 6; ++k) stamps[8 + k] = ss.v[k];
    }
  }
}

template <int NT, int R, int W, int MODE, bool STAMP = false>
__global__ __launch_bounds__(NT) void panel_kernel(double* __restrict__ P, int64_t ldp, int m,
                                                   int w, int row0, int* __restrict__ piv,
                                                   int* __restrict__ info,
                                                   unsigned long long* __restrict__ stamps,
                                                   int* __restrict__ pairs) {
  __shared__ PanelLds<W> sh;
  panel_body<NT, R, W, MODE, STAMP>(P, ldp, m, w, row0, piv, info, stamps, pairs, sh);
}

// ---- fused step kernel -----------------------------------------------------
// One launch per blocked-LU step j (the right-looking sweep with lookahead
// folded into a single grid, so no cross-stream events are needed):
//   workgroup 0      : applies step j-1 (row movement, TRSM, rank-wp GEMM) to
//                      panel j's own column strip, then factors panel j;
//   workgroups 1..   : apply step j-1 to one 16-column strip each of the
//                      columns right of panel j (b included).
// The wide update of step j-1 therefore runs on ~n/16 CUs underneath the
// single-CU panel factorisation of step j.  Every workgroup owns whole
// columns, so the row interchanges need no cross-workgroup ordering.
constexpr int kStripCols = 16;
constexpr int kStripMaxW = 16;

struct NarrowArgs {
  const double* C;  // strip: A + kp*lda + k (rows relative to kp)
  int64_t ldc;
  int ncols;        // strip width (next panel's w)
  const double* L;  // step-j panel, column-major (ld ldl)
  int64_t ldl;
  int wp;           // step-j panel width
  int m;            // n - kp
  const int* pairs; // step-j row movement
  double* out;      // buffer, column-major (rows relative to kp), ld ldo
  int64_t ldo;
};

struct StepArgs {
  double* A;
  int64_t lda;
  int n;
  int kp, wp;              // previous step (wp = 0: none)
  const int* pairs_prev;   // its net row movement (relative to kp)
  int k, w;                // this step's panel (w = 0: none)
  int* piv;
  int* info;
  int* pairs;              // this step's row movement (out)
  int wide_c0;             // first column of the wide strips
  unsigned long long* stamps;  // diagnostics (STAMP builds): realtime per phase
  int io;                      // panel IO: 0 LDS-staged, 1 direct
  const double* buf;           // narrow-kernel output (rows rel kp, column-major, ld ldL) or null
  double* lout;                // this step's factored panel, column-major (ld ldL)
  const double* lprev;         // the previous step's, same layout
  int ldL;                     // >= NT * R of every step (padding rows absorb the
                               // unconditional early stores)
  // fused narrow update (nflags != null): nnar trailing workgroups apply
  // THIS step to the next panel's strip (nar, as lu_narrow would) once the
  // first wide workgroup has updated that strip (nflags[0]) and workgroup 0
  // has factored the panel (nflags[1]) -- no separate narrow launch
  unsigned* nflags;
  int nwide, nnar;
  NarrowArgs nar;
};


// Panel IO of the fused step: 2 = every coalesced load in flight at once +
// LDS transpose, LDS-staged coalesced stores (1 = direct 16-byte register
// loads/stores, 0 = LDS-staged passes one slot at a time measured within
// noise of it, profiles/headline_2048_r4.md).
int panel_io_mode() { return 2; }

__device__ __forceinline__ unsigned long long realtime_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

struct alignas(16) StripLds {
  double g[2 * kStripMaxW][kStripCols];   // gathered source rows
  double x[kStripMaxW][kStripCols];       // top rows -> U12
  double l11[kStripMaxW][kStripMaxW];     // unit lower triangle of the previous panel
  int pr[1 + 4 * kStripMaxW];
};

// Apply a finished panel (rows [0, m) relative to its top, width wp, net row
// movement `pairs`; L column-major with leading dimension ldl, final row
// order) to an ncols <= 16 column strip C: swap, U12 = L11^-1 A12,
// A22 -= L21 U12 on the fp64 matrix cores.  Whole workgroup (NT = 512).
// One forward-substitution step of the DPP-row TRSM (see strip_update).
template <int I>
__device__ __forceinline__ void trsm_dpp_step(double& x, const double (&lrow)[kStripMaxW], int j) {
  const uint64_t bits = (uint64_t)__double_as_longlong(x);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(bits >> 32), 0x150 + I, 0xf, 0xf, false);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)bits, 0x150 + I, 0xf, 0xf, false);
  const double xi = __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
  x = (j > I) ? fma(-lrow[I], xi, x) : x;
}

template <int... I>
__device__ __forceinline__ void trsm_dpp_steps(double& x, const double (&lrow)[kStripMaxW], int j,
                                               std::integer_sequence<int, I...>) {
  (trsm_dpp_step<I>(x, lrow, j), ...);
}

template <int NT, bool STAMP = false>
__device__ __forceinline__ void strip_update(double* __restrict__ C, int64_t ldc, int ncols,
                                             const double* __restrict__ L, int64_t ldl, int wp,
                                             int m, const int* __restrict__ pairs, StripLds& sh,
                                             unsigned long long* ts = nullptr) {
  static_assert(NT == 2 * kStripMaxW * kStripCols, "one thread per (pair, column)");
  auto mark = [&](int i) {
    if constexpr (STAMP) ts[i] = realtime_now();
  };
  const int t = threadIdx.x;
  const int c = t & (kStripCols - 1);
  const int e = t >> 4;
  const bool colok = c < ncols;
  // U12 rows and the updated block are stored write-through (dev::store_wt)
  const __amdgpu_buffer_rsrc_t crs = dev::buffer_rsrc(C, ((uint64_t)(m - 1) * ldc + kStripCols) * 8);
  const int cc = min(c, ncols - 1);  // clamped column: every load below is unconditional
  if (t < 1 + 4 * kStripMaxW) {
    const int np = pairs[0];
    sh.pr[t] = dev::load_sel(pairs + t, t == 0 || t <= 2 * np);
  }
  if (t < kStripMaxW * kStripMaxW) {
    const int r = t / kStripMaxW, q = t % kStripMaxW;
    const int rc = min(r, wp - 1), qc = min(q, wp - 1);
    sh.l11[r][q] = dev::load_sel(L + (int64_t)qc * ldl + rc, q < r && r < wp);
  }
  const double top = dev::load_sel(C + (int64_t)min(e, wp - 1) * ldc + cc, e < wp && colok);
  __syncthreads();
  mark(0);
  const int np = sh.pr[0];
  // every source and every top row is read before anything is written
  {
    const int src = sh.pr[2 + 2 * min(e, 4 * kStripMaxW / 2 - 1)];  // 0 beyond np: row 0
    const double gv = C[(int64_t)src * ldc + cc];
    if (e < np && colok) sh.g[e][c] = gv;
  }
  if (e < kStripMaxW) sh.x[e][c] = top;
  __syncthreads();
  mark(1);
  if (e < np && colok) {
    const int d = sh.pr[1 + 2 * e];
    if (d < wp) sh.x[d][c] = sh.g[e][c];
    else C[(int64_t)d * ldc + c] = sh.g[e][c];
  }
  __syncthreads();
  mark(2);
  if (t < kStripCols * kStripMaxW) {  // forward substitution: DPP row = one column
    // lane j of 16-lane row c holds x[j][c]; x[i][c] is broadcast to the row
    // with DPP row_newbcast:i, so the 16-step chain has no LDS round trips
    const int cc = t >> 4, j = t & 15;
    double x = sh.x[j][cc];
    double lrow[kStripMaxW];
#pragma unroll
    for (int i = 0; i < kStripMaxW; ++i) lrow[i] = sh.l11[j][i];
    trsm_dpp_steps(x, lrow, j, std::make_integer_sequence<int, kStripMaxW>{});
    sh.x[j][cc] = x;
    if (j < wp && cc < ncols) dev::store_wt(crs, (uint32_t)(((int64_t)j * ldc + cc) * 8), x);
  }
  __syncthreads();
  mark(3);
  // rank-wp update of rows [wp, m): v_mfma_f64_16x16x4 per 16-row block,
  // 4 blocks per wave in flight.  K is permuted so each lane reads 4
  // consecutive multipliers (two 16-byte loads): MFMA kk, lane group q covers
  // k = 4q + kk, and the B operand is read with the same permutation.
  const int lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  constexpr int kWaves = NT / 64;
  constexpr int kBatch = 4;
  double b[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) b[kk] = sh.x[4 * q + kk][r16];
  const bool ccol = r16 < ncols;
  const int nblk = (m - wp + 15) >> 4;
  for (int b0 = wave; b0 < nblk; b0 += kWaves * kBatch) {
    dev::d4 acc[kBatch];
    double la[kBatch][4];
#pragma unroll
    for (int s = 0; s < kBatch; ++s) {
      const int blk = b0 + kWaves * s;
      const int rbase = wp + 16 * blk;
      const int lrow = rbase + r16;
      // clamped rows / columns: unconditional loads, selects afterwards
      const bool okb = blk < nblk && lrow < m;
      const double* lp = L + min(lrow, m - 1);  // column-major: lanes r16 coalesce
#pragma unroll
      for (int e = 0; e < 4; ++e)
        la[s][e] = dev::load_sel(lp + (int64_t)min(4 * q + e, wp - 1) * ldl, okb && 4 * q + e < wp);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + q + 4 * r;
        acc[s][r] = dev::load_sel(C + (int64_t)min(row, m - 1) * ldc + min(r16, ncols - 1),
                                  blk < nblk && row < m && ccol);
      }
    }
#pragma unroll
    for (int s = 0; s < kBatch; ++s)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double a = (4 * q + kk < wp) ? -la[s][kk] : 0.0;
        acc[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[kk], acc[s], 0, 0, 0);
      }
#pragma unroll
    for (int s = 0; s < kBatch; ++s) {
      const int blk = b0 + kWaves * s;
      const int rbase = wp + 16 * blk;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rbase + q + 4 * r;
        if (blk < nblk && row < m && ccol)
          dev::store_wt(crs, (uint32_t)(((int64_t)row * ldc + r16) * 8), acc[s][r]);
      }
    }
  }
  mark(4);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // strip complete before any reader
  mark(5);
}

// ---- narrow kernel ------------------------------------------------------------
// Step j applied to the NEXT panel's column strip, spread over ceil(m/64)
// workgroups (one 64-row slice each: 2048: 3.96 ms vs 3.99 with 128 and 4.03
// with 256-row slices) instead of serialising it on the panel
// workgroup.  A is only read; the updated strip (rows relative to the step-j
// panel top, U12 rows first) goes to a side buffer that the next panel loads
// directly, so the row interchanges need no cross-workgroup ordering.
constexpr int kNarrowRows = 64;


// Coherent loads for the fused narrow update (StepArgs::nflags): the strip,
// the panel and its row movement were written by other workgroups of the
// same launch (possibly on other XCDs) with write-through stores, so they are
// read with agent-scope (sc1) loads; the narrow kernel reads plain.
template <bool COH, typename T>
__device__ __forceinline__ T ldc(const T* p) {
  if constexpr (COH) {
    if constexpr (sizeof(T) == 8) {
      const unsigned long long v =
          __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return __builtin_bit_cast(T, v);
    } else {
      const unsigned v = __hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      return __builtin_bit_cast(T, v);
    }
  } else {
    return *p;
  }
}
template <bool COH, typename T>
__device__ __forceinline__ T ldc_sel(const T* p, bool ok) {
  const T v = ldc<COH>(p);
  return ok ? v : T(0);
}

constexpr int kNarrowMaxRows = 128;
struct alignas(16) NarrowLds {
  double x[kStripMaxW][kStripCols];
  double l11[kStripMaxW][kStripMaxW];
  int pr[1 + 4 * kStripMaxW];
  int srcmap[kNarrowMaxRows];
};

// Rows [r0, r0 + 16 * NT / 64) of the narrow update (one 16-row MFMA block
// per wave), NT threads.
template <int NT, bool COH>
__device__ __forceinline__ void narrow_body(const NarrowArgs& g, int r0, NarrowLds& sh) {
  constexpr int kRows = 16 * (NT / 64);
  static_assert(kRows <= kNarrowMaxRows, "narrow slice");
  const int t = threadIdx.x;
  const __amdgpu_buffer_rsrc_t ors = dev::buffer_rsrc(g.out, (uint64_t)kStripCols * g.ldo * 8);
  const int r1 = min(r0 + kRows, g.m);
  const int wp = g.wp, ncols = g.ncols;
  const int lane = t & 63, wave = t >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const bool ccol = r16 < ncols;
  const int a0 = max(r0, wp);
  const int nblk = (r1 - a0 + 15) >> 4;  // <= NT / 64
  // Round trip 1 — everything that does not depend on the row movement is in
  // flight together: pairs, L11, the top rows, this slice's multipliers and
  // its strip rows at their own positions (unmoved rows: all but <= 2w).
  dev::d4 acc;
  double la[4];
  if (t < 256) {
    const int rr = t >> 4, cc = t & 15;
    // the whole pair slot in one round trip (entries past 2 * pairs[0] are
    // never used), not pairs[0] first and the pairs behind it
    if (t < 1 + 4 * kStripMaxW) sh.pr[t] = ldc<COH>(g.pairs + t);
    sh.l11[rr][cc] = ldc_sel<COH>(g.L + (int64_t)min(cc, wp - 1) * g.ldl + min(rr, wp - 1), cc < rr && rr < wp);
    sh.x[rr][cc] = ldc_sel<COH>(g.C + (int64_t)min(rr, wp - 1) * g.ldc + min(cc, ncols - 1), rr < wp && cc < ncols);
  }
  if (t < kRows) sh.srcmap[t] = r0 + t;
  const int rbase = a0 + 16 * wave;
  {
    const int lrow = rbase + r16;
    const bool okb = wave < nblk && lrow < r1;
    const double* lp = g.L + min(lrow, r1 - 1);  // column-major L
#pragma unroll
    for (int e = 0; e < 4; ++e)
      la[e] = ldc_sel<COH>(lp + (int64_t)min(4 * q + e, wp - 1) * g.ldl, okb && 4 * q + e < wp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = rbase + q + 4 * r;
      const int rowc = min(max(row, r0), r1 - 1);
      acc[r] = ldc_sel<COH>(g.C + (int64_t)rowc * g.ldc + min(r16, ncols - 1), wave < nblk && row < r1 && ccol);
    }
  }
  __syncthreads();
  const int np = sh.pr[0];
  // round trip 2: post-swap top rows; source rows of this slice's permuted rows
  for (int idx = t; idx < np * kStripCols; idx += NT) {
    const int e = idx >> 4, cc = idx & 15;
    const int d = sh.pr[1 + 2 * e];
    if (d < wp) sh.x[d][cc] = ldc_sel<COH>(g.C + (int64_t)sh.pr[2 + 2 * e] * g.ldc + min(cc, ncols - 1), cc < ncols);
  }
  if (t < np) {
    const int d = sh.pr[1 + 2 * t];
    if (d >= r0 && d < r1) sh.srcmap[d - r0] = sh.pr[2 + 2 * t];
  }
  __syncthreads();
  // the moved rows of this slice re-read their source (in flight under the TRSM)
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rbase + q + 4 * r;
    const int rowc = min(max(row, r0), r1 - 1);
    const int src = sh.srcmap[rowc - r0];
    if (src != rowc && wave < nblk && row < r1 && ccol) acc[r] = ldc<COH>(g.C + (int64_t)src * g.ldc + r16);
  }
  if (t < 256) {  // U12 = L11^-1 x: DPP row = one column
    const int cc = t >> 4, j = t & 15;
    double xv = sh.x[j][cc];
    double lrow[kStripMaxW];
#pragma unroll
    for (int i = 0; i < kStripMaxW; ++i) lrow[i] = sh.l11[j][i];
    trsm_dpp_steps(xv, lrow, j, std::make_integer_sequence<int, kStripMaxW>{});
    sh.x[j][cc] = xv;
    if (r0 == 0 && j < wp) dev::store_wt(ors, (uint32_t)(((int64_t)cc * g.ldo + j) * 8), xv);
  }
  __syncthreads();
  // rows [max(r0, wp), r1): out[r] = A[src(r)] - L[r] U12 (MFMA, K permuted)
  double b[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) b[kk] = sh.x[4 * q + kk][r16];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const double a = (4 * q + kk < wp) ? -la[kk] : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[kk], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = rbase + q + 4 * r;
    if (wave < nblk && row < r1) dev::store_wt(ors, (uint32_t)(((int64_t)r16 * g.ldo + row) * 8), acc[r]);
  }
}

__global__ __launch_bounds__(256) void narrow_kernel(NarrowArgs g) {
  __shared__ NarrowLds sh;
  narrow_body<256, false>(g, blockIdx.x * kNarrowRows, sh);
}

// Hand-off inside one step launch (write-through recipe, rlu.hip): every
// wave's stores drain, barrier, one lane sets the flag; the waiting workgroup
// polls it relaxed (bounded: 200 ms, then code 11 in info[1]) and reads the
// payload with sc1 loads.
__device__ __forceinline__ void publish_flag(unsigned* f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool wait_flags(unsigned* f, bool strip, int* info, NarrowLds& sh) {
  if (threadIdx.x == 0) {
    int ok = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = strip ? 0 : 1; i < 2 && ok; ++i) {
      while (__hip_atomic_load(f + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // 200 ms at 100 MHz
          __hip_atomic_store(info + 1, 11, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    sh.srcmap[0] = ok;
  }
  __syncthreads();
  const bool ok = sh.srcmap[0] != 0;
  __syncthreads();  // srcmap is reused by the slice
  return ok;
}

template <int NT, int R, int W, int MODE, bool STAMP = false>
__global__ __launch_bounds__(NT) void step_kernel(StepArgs g) {
  __shared__ PanelLds<W> sh;
  StripLds& ss = *reinterpret_cast<StripLds*>(g_panel_dyn_lds);
  const bool has_panel = g.w > 0;
  const int64_t lda = g.lda;
  unsigned long long t0 = 0, t1 = 0;
  __shared__ unsigned long long sts[8];
  if constexpr (STAMP) t0 = realtime_now();
  if (has_panel && blockIdx.x == 0 && g.buf != nullptr) {
    // step j-1 was already applied to this strip by the narrow kernel: its
    // U12 rows go to A, the panel rows are read straight from the buffer
    {
      const int r = threadIdx.x >> 4, c = threadIdx.x & 15;
      if (r < g.wp && c < g.w)
        g.A[(int64_t)(g.kp + r) * lda + g.k + c] = g.buf[(int64_t)c * g.ldL + r];
    }
    if constexpr (STAMP) t1 = realtime_now();
    panel_body<NT, R, W, MODE, STAMP>(g.A + (int64_t)g.k * lda + g.k, lda, g.n - g.k, g.w, g.k,
                                      g.piv + g.k, g.info, STAMP ? g.stamps + 700 : nullptr,
                                      g.pairs, sh, g.io, g.buf + g.wp, g.ldL, g.lout, g.ldL, true);
    if (g.nflags) publish_flag(g.nflags + 1);
    if constexpr (STAMP) {
      __syncthreads();
      if (threadIdx.x == 0) {
        g.stamps[0] = t0;
        g.stamps[1] = t1;
        g.stamps[2] = realtime_now();
      }
    }
    return;
  }
  if (has_panel && blockIdx.x == 0) {
    if (g.wp > 0) {
      strip_update<NT, STAMP>(g.A + (int64_t)g.kp * lda + g.k, lda, g.w, g.lprev, g.ldL, g.wp,
                              g.n - g.kp, g.pairs_prev, ss, sts);
      __syncthreads();  // strip writes visible to the panel's loads (same CU)
    }
    if constexpr (STAMP) t1 = realtime_now();
    panel_body<NT, R, W, MODE, false>(g.A + (int64_t)g.k * lda + g.k, lda, g.n - g.k, g.w, g.k,
                                      g.piv + g.k, g.info, nullptr, g.pairs, sh, g.io, nullptr, 0,
                                      g.lout, g.ldL);
    if (g.nflags) publish_flag(g.nflags + 1);
    if constexpr (STAMP) {
      __syncthreads();
      if (threadIdx.x == 0) {
        g.stamps[0] = t0;
        g.stamps[1] = t1;
        g.stamps[2] = realtime_now();
        for (int i = 0; i < 6; ++i) g.stamps[600 + i] = sts[i];
      }
    }
    return;
  }
  const int wb = (int)(blockIdx.x - (has_panel ? 1 : 0));
  if (g.nflags && wb >= g.nwide) {  // fused narrow slice
    NarrowLds& nl = *reinterpret_cast<NarrowLds*>(g_panel_dyn_lds);
    if (!wait_flags(g.nflags, g.wp > 0, g.info, nl)) return;
    narrow_body<NT, true>(g.nar, (wb - g.nwide) * 16 * (NT / 64), nl);
    return;
  }
  const int c0 = g.wide_c0 + kStripCols * wb;
  const int ncols = min(kStripCols, g.n + 1 - c0);
  if (ncols <= 0) return;
  strip_update<NT>(g.A + (int64_t)g.kp * lda + c0, lda, ncols, g.lprev, g.ldL, g.wp, g.n - g.kp,
                   g.pairs_prev, ss);
  if (g.nflags && wb == 0) publish_flag(g.nflags);  // the next panel's strip is up to date
  if constexpr (STAMP) {
    __syncthreads();
    if (threadIdx.x == 0) {
      g.stamps[8 + 2 * wb] = t0;
      g.stamps[9 + 2 * wb] = realtime_now();
    }
  }
}

template <int NT, int R, int W>
int launch_step(const StepArgs& a, int mode, unsigned blocks, hipStream_t s) {
  constexpr size_t stage = Panel<NT, R, W, 1, false>::stage_bytes();
  constexpr size_t lds = stage > sizeof(StripLds) ? stage : sizeof(StripLds);
  if (mode == GELIM_PIVOT_PARTIAL)
    hipLaunchKernelGGL((step_kernel<NT, R, W, 1>), dim3(blocks), dim3(NT), lds, s, a);
  else
    hipLaunchKernelGGL((step_kernel<NT, R, W, 0>), dim3(blocks), dim3(NT), lds, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

template <int NT, int R, int W>
int launch_panel(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode, int* piv,
                 int* info, int* pairs, hipStream_t s) {
  constexpr size_t lds = Panel<NT, R, W, 1, false>::stage_bytes();
  if (mode == GELIM_PIVOT_PARTIAL)
    hipLaunchKernelGGL((panel_kernel<NT, R, W, 1>), dim3(1), dim3(NT), lds, s, P, ldp, (int)m,
                       (int)w, (int)row0, piv, info, nullptr, pairs);
  else
    hipLaunchKernelGGL((panel_kernel<NT, R, W, 0>), dim3(1), dim3(NT), lds, s, P, ldp, (int)m,
                       (int)w, (int)row0, piv, info, nullptr, pairs);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// Widest register panel for m rows (R x W <= 64 doubles per lane at 512
// threads: 256 KiB of panel on one CU).
int64_t panel_width_for(int64_t m) {
  if (m <= 2048) return 16;
  if (m <= 4096) return 8;
  if (m <= 8192) return 4;
  if (m <= 16384) return 2;
  return 0;
}

int panel_factor(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode, int* piv,
                 int* info, hipStream_t s, int* pairs) {
  if (m <= 0 || w <= 0 || w > m) return GELIM_FAIL(GELIM_E_ARG, "panel: bad m/w");
  if (m <= 512 && w <= 16) return launch_panel<512, 1, 16>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  if (m <= 1024 && w <= 16) return launch_panel<512, 2, 16>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  if (m <= 2048 && w <= 16) return launch_panel<512, 4, 16>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  if (m <= 4096 && w <= 8) return launch_panel<512, 8, 8>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  if (m <= 8192 && w <= 4) return launch_panel<512, 16, 4>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  if (m <= 16384 && w <= 2) return launch_panel<512, 32, 2>(P, ldp, m, w, row0, mode, piv, info, pairs, s);
  return GELIM_FAIL(GELIM_E_ARG, "panel: m=" + std::to_string(m) + " w=" + std::to_string(w) +
                                     " exceeds the register-resident panel");
}

// One fused step of the blocked LU (see step_kernel).  (kp, wp): previous
// panel (wp = 0 for the first step); (k, w): this step's panel (w = 0 for the
// closing step that only finishes the previous update).
// Rows of the column-major panel buffers (lout / lprev of lu_step): >= NT * R
// of the first (largest) step, so every early column store lands in bounds.
// Steps of <= 1536 rows run on 3 rows per lane (3.76 -> 3.73 ms per 2048
// solve, profiles/headline_2048_r4.md).

int64_t lu_panel_buffer_ld(int64_t n) {
  int64_t r = 512;
  while (r < n) r *= 2;
  return r;
}

int lu_step(double* A, int64_t lda, int64_t n, int64_t kp, int64_t wp, const int* pairs_prev,
            int64_t k, int64_t w, int mode, int* piv, int* info, int* pairs, hipStream_t s,
            const double* buf, double* lout, const double* lprev, int64_t ldL, unsigned* nflags = nullptr,
            double* nbuf = nullptr, int64_t nk = 0, int64_t nw = 0) {
  if (wp > kStripMaxW || w > 16) return GELIM_FAIL(GELIM_E_ARG, "lu_step: panel wider than 16");
  if (ldL < lu_panel_buffer_ld(n) || (w > 0 && !lout) || (wp > 0 && !lprev))
    return GELIM_FAIL(GELIM_E_ARG, "lu_step: panel buffers missing or too small");
  StepArgs a{A, lda, (int)n, (int)kp, (int)wp, pairs_prev, (int)k, (int)w, piv, info, pairs, 0,
             nullptr, panel_io_mode(), (w > 0 && wp > 0) ? buf : nullptr, lout, lprev, (int)ldL};
  // w = 0: closing launch, step (kp, wp) applied to every column from k on
  // (k = n: just b; the hybrid schedule closes at its split column)
  const int64_t c0 = (w > 0) ? k + w : k;
  a.wide_c0 = (int)c0;
  const int64_t nwide = (wp > 0) ? (n + 1 - c0 + kStripCols - 1) / kStripCols : 0;
  const int64_t m = n - (w > 0 ? k : kp);
  a.nflags = nullptr;
  a.nwide = (int)nwide;
  a.nnar = 0;
  if (nflags && w > 0 && nw > 0) {
    // fused narrow update of the next panel's strip [nk, nk + nw) (lu_narrow's
    // arguments), one 128-row slice per trailing workgroup (NT = 512)
    if (nw > kStripCols || nk != k + w || !nbuf)
      return GELIM_FAIL(GELIM_E_ARG, "lu_step: fused narrow strip must follow the panel, width <= 16");
    a.nflags = nflags;
    a.nnar = (int)((m + 127) / 128);
    a.nar = NarrowArgs{A + k * lda + nk, lda, (int)nw, lout, ldL, (int)w, (int)m, pairs, nbuf, ldL};
  }
  const unsigned blocks = (unsigned)(nwide + (w > 0 ? 1 : 0) + a.nnar);
  if (blocks == 0) return GELIM_OK;
  if (m <= 512 && w <= 16) return launch_step<512, 1, 16>(a, mode, blocks, s);
  if (m <= 1024 && w <= 16) return launch_step<512, 2, 16>(a, mode, blocks, s);
  // 3 rows per lane below 1536 rows: the column loop is VALU-issue bound and
  // its per-row work shrinks by a quarter (round 4: 3.76 -> 3.73 ms at 2048)
  if (m <= 1536 && w <= 16) return launch_step<512, 3, 16>(a, mode, blocks, s);
  if (m <= 2048 && w <= 16) return launch_step<512, 4, 16>(a, mode, blocks, s);
  if (m <= 4096 && w <= 8) return launch_step<512, 8, 8>(a, mode, blocks, s);
  if (m <= 8192 && w <= 4) return launch_step<512, 16, 4>(a, mode, blocks, s);
  if (m <= 16384 && w <= 2) return launch_step<512, 32, 2>(a, mode, blocks, s);
  return GELIM_FAIL(GELIM_E_ARG, "lu_step: m=" + std::to_string(m) + " w=" + std::to_string(w) +
                                     " exceeds the register-resident panel");
}

// Step (kp, wp) applied to the next panel's strip [k, k + w) into buf
// (rows relative to kp, column-major, ld ldL: 16 x ldL doubles); L is step
// kp's factored panel (column-major, ld ldL) from lu_step.
int lu_narrow(double* A, int64_t lda, int64_t n, int64_t kp, int64_t wp, const int* pairs,
              int64_t k, int64_t w, double* buf, hipStream_t s, const double* L, int64_t ldL) {
  if (wp > kStripMaxW || w > kStripCols) return GELIM_FAIL(GELIM_E_ARG, "lu_narrow: width > 16");
  const int64_t m = n - kp;
  NarrowArgs a{A + kp * lda + k, lda, (int)w, L, ldL, (int)wp, (int)m, pairs, buf, ldL};
  hipLaunchKernelGGL(narrow_kernel, dim3((unsigned)((m + kNarrowRows - 1) / kNarrowRows)), dim3(256), 0,
                     s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace gelim

extern "C" int gelim_gpu_panel_factor(double* dP, int64_t ldp, int64_t m, int64_t w, int64_t row0,
                                      int pivot, int32_t* dpiv, int32_t* dinfo, void* stream) {
  return gelim::panel_factor(dP, ldp, m, w, row0, pivot, dpiv, dinfo, (hipStream_t)stream, nullptr);
}

// Diagnostic: run the stamped panel kernel on an m x 16 panel (w columns
// factored) and return {t_load, t_steps, t_store, total} in shader cycles,
// then the phase boundaries of column step 4 relative to its start.
extern "C" int gelim_debug_panel_stamps(int64_t m, int64_t w, unsigned long long* out) {
  using namespace gelim;
  double* P = nullptr;
  int *piv = nullptr, *info = nullptr;
  unsigned long long* st = nullptr;
  HIP_TRY(hipMalloc((void**)&P, sizeof(double) * m * 16));
  HIP_TRY(hipMalloc((void**)&piv, sizeof(int) * 64));
  HIP_TRY(hipMalloc((void**)&info, 16));
  HIP_TRY(hipMalloc((void**)&st, 256));
  HIP_TRY(hipMemset(st, 0, 256));
  std::vector<double> h(m * 16);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 997.0 - 0.5;
  HIP_TRY(hipMemcpy(P, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(info, 0, 16));
  constexpr size_t lds = Panel<512, 4, 16, 1, true>::stage_bytes();
  for (int rep = 0; rep < 3; ++rep) {
    if (m <= 512)
      hipLaunchKernelGGL((panel_kernel<512, 1, 16, 1, true>), 1, 512, lds, 0, P, 16, (int)m,
                         (int)w, 0, piv, info, st, nullptr);
    else if (m <= 1024)
      hipLaunchKernelGGL((panel_kernel<512, 2, 16, 1, true>), 1, 512, lds, 0, P, 16, (int)m,
                         (int)w, 0, piv, info, st, nullptr);
    else
      hipLaunchKernelGGL((panel_kernel<512, 4, 16, 1, true>), 1, 512, lds, 0, P, 16, (int)m,
                         (int)w, 0, piv, info, st, nullptr);
    HIP_TRY(hipDeviceSynchronize());
  }
  unsigned long long hs[32];
  HIP_TRY(hipMemcpy(hs, st, 256, hipMemcpyDeviceToHost));
  out[0] = hs[1] - hs[0];
  out[1] = hs[2] - hs[1];
  out[2] = hs[3] - hs[2];
  out[3] = hs[3] - hs[0];
  for (int k = 1; k <= 5; ++k) out[3 + k] = hs[8 + k] >= hs[8] ? hs[8 + k] - hs[8] : 0;
  (void)hipFree(P);
  (void)hipFree(piv);
  (void)hipFree(info);
  (void)hipFree(st);
  return GELIM_OK;
}

extern "C" int64_t gelim_gpu_panel_max_rows(int64_t w) {
  if (w <= 2) return 16384;
  if (w <= 4) return 8192;
  if (w <= 8) return 4096;
  if (w <= 16) return 2048;
  return 0;
}

// Diagnostic: factor a random n x (n+1) system up to step j (fused schedule,
// 16-wide panels, n <= 2048), then run step j with realtime stamps.  out[0..2]
// = workgroup 0 {prologue, panel} in 10 ns ticks; out[3] = slowest wide
// workgroup, out[4] = median wide workgroup, out[5] = wide count.
extern "C" int gelim_debug_step_stamps(int64_t n, int64_t j, double* out) {
  using namespace gelim;
  if (n > 2048 || j < 1 || 16 * j >= n) return GELIM_FAIL(GELIM_E_ARG, "debug_step_stamps: bad n/j");
  const int64_t lda = (n + 1 + 7) / 8 * 8;
  double* A = nullptr;
  int *piv = nullptr, *info = nullptr, *pairs = nullptr;
  unsigned long long* st = nullptr;
  HIP_TRY(hipMalloc((void**)&A, sizeof(double) * n * lda));
  HIP_TRY(hipMalloc((void**)&piv, sizeof(int) * (n + 64)));
  HIP_TRY(hipMalloc((void**)&info, 16));
  HIP_TRY(hipMalloc((void**)&pairs, sizeof(int) * 72 * (n / 16 + 2)));
  HIP_TRY(hipMalloc((void**)&st, sizeof(unsigned long long) * 1024));
  HIP_TRY(hipMemset(st, 0, sizeof(unsigned long long) * 1024));
  HIP_TRY(hipMemset(info, 0, 16));
  std::vector<double> h(n * lda, 0.0);
  for (int64_t r = 0; r < n; ++r)
    for (int64_t c = 0; c <= n; ++c)
      h[r * lda + c] = (double)(((r * 7919 + c * 104729) * 2654435761ull) % 2000) / 1000.0 - 1.0;
  HIP_TRY(hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  double* sbuf = nullptr;
  const int64_t ldL = lu_panel_buffer_ld(n);
  HIP_TRY(hipMalloc((void**)&sbuf, sizeof(double) * 16 * ldL));
  double* lbuf = nullptr;
  HIP_TRY(hipMalloc((void**)&lbuf, sizeof(double) * 2 * 16 * ldL));
  auto lb = [&](int64_t i) { return lbuf + (i & 1) * 16 * ldL; };
  const bool nar = true;
  for (int64_t i = 0; i < j; ++i) {
    GELIM_TRY(lu_step(A, lda, n, i ? 16 * (i - 1) : 0, i ? 16 : 0, i ? pairs + (i - 1) * 72 : nullptr,
                      16 * i, 16, GELIM_PIVOT_PARTIAL, piv, info, pairs + i * 72, 0,
                      nar ? sbuf : nullptr, lb(i), i ? lb(i - 1) : nullptr, ldL));
    if (nar)
      GELIM_TRY(lu_narrow(A, lda, n, 16 * i, 16, pairs + i * 72, 16 * (i + 1), 16, sbuf, 0, lb(i), ldL));
  }
  StepArgs a{A, lda, (int)n, (int)(16 * (j - 1)), 16, pairs + (j - 1) * 72, (int)(16 * j), 16,
             piv, info, pairs + j * 72, (int)(16 * j + 16), st, panel_io_mode(),
             nar ? sbuf : nullptr, lb(j), lb(j - 1), (int)ldL};
  const int64_t m = n - 16 * j;
  const unsigned nwide = (unsigned)((n + 1 - (16 * j + 16) + 15) / 16);
  constexpr size_t lds = Panel<512, 4, 16, 1, false>::stage_bytes();
  if (m <= 512)
    hipLaunchKernelGGL((step_kernel<512, 1, 16, 1, true>), nwide + 1, 512, lds, 0, a);
  else if (m <= 1024)
    hipLaunchKernelGGL((step_kernel<512, 2, 16, 1, true>), nwide + 1, 512, lds, 0, a);
  else
    hipLaunchKernelGGL((step_kernel<512, 4, 16, 1, true>), nwide + 1, 512, lds, 0, a);
  HIP_TRY(hipDeviceSynchronize());
  std::vector<unsigned long long> hs(1024);
  HIP_TRY(hipMemcpy(hs.data(), st, 8 * 1024, hipMemcpyDeviceToHost));
  const unsigned long long base = hs[0];
  out[0] = (double)(hs[1] - base);
  out[1] = (double)(hs[2] - hs[1]);
  out[2] = (double)(hs[2] - base);
  std::vector<double> wd;
  for (unsigned b = 0; b < nwide && 9 + 2 * b < 1024; ++b) wd.push_back((double)(hs[9 + 2 * b] - base));
  std::sort(wd.begin(), wd.end());
  out[3] = wd.empty() ? 0 : wd.back();
  out[4] = wd.empty() ? 0 : wd[wd.size() / 2];
  out[5] = (double)wd.size();
  for (int i = 0; i < 6; ++i) out[6 + i] = hs[600 + i] ? (double)(hs[600 + i] - base) : 0.0;
  // panel internals (s_memtime cycles -> 10 ns ticks at 2.4 GHz): load, steps, store
  out[12] = (double)(hs[701] - hs[700]) / 24.0;
  out[13] = (double)(hs[702] - hs[701]) / 24.0;
  out[14] = (double)(hs[703] - hs[702]) / 24.0;
  // store phase split: reconstruction+drain, barrier, dest, fix-ups+end
  out[15] = (double)(hs[704] - hs[702]) / 24.0;
  out[16] = (double)(hs[705] - hs[704]) / 24.0;
  out[17] = (double)(hs[706] - hs[705]) / 24.0;
  out[18] = (double)(hs[703] - hs[706]) / 24.0;
  out[19] = (double)(hs[707] - hs[702]) / 24.0;  // reconstruction alone (wave 0)
  (void)hipFree(sbuf);
  (void)hipFree(lbuf);
  (void)hipFree(A);
  (void)hipFree(piv);
  (void)hipFree(info);
  (void)hipFree(pairs);
  (void)hipFree(st);
  return GELIM_OK;
}
