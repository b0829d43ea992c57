// The 32-column multi-workgroup leaf of the wide-panel LU (biglu.hip): one
// m x 32 panel factored with partial pivoting (or the reference's zero
// rule) by P participant workgroups of NWV waves.  Template code shared by
// the instantiation units leaf_w*.hip (split so the heavily unrolled
// variants compile in parallel); the host dispatch is big::leaf_factor.
//
// What it computes: the reference's getPivot + elimination sweep
// (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:123-182; the strict
// '>' of Pthreads/Version-1/gauss_external_input.c:130-134 = ties to the
// lowest row) on 32 columns, LAPACK row order.
//
// Layout: participant p = blockIdx.x owns rows [p * NWV * 64 R, +NWV * 64 R);
// wave w of it the 64 R rows from (p * NWV + w) * 64 R, lane l the rows
// base + l + 64 i (i < R) -- 32 columns each, register resident.  Shapes
// (NWV x R): 1 x 2 by default, 1 x 1, 1 x 4, 2 x 2, 4 x 1, 4 x 4
// (biglu.hip leaf_shape).
//
// Per column J:
//  1. every lane's best live row, the wave's arg-max (DPP, one ballot);
//  2. NWV > 1: the waves of a participant merge their candidates in LDS
//     behind ONE workgroup barrier (candidate row + key, parity-buffered);
//     one wave then publishes the participant's winner to global memory as
//     LW data-tagged 16-byte sc1 granules {value, row, tag} plus a key
//     granule -- so the cross-CU exchange has P = m / (256 NWV) parties
//     instead of m / 256;
//  3. every wave polls the P key granules (and, for P <= 32, every
//     candidate row in the same sweep) with sc1 loads until all carry the tag,
//     picks the global winner and takes its row into a wave-private LDS line;
//  4. multipliers, the rank-1 update of column J+1 now and of the rest under
//     the next exchange.
// Granules are double-buffered by column parity and by leaf set (leaf
// counter & 1) and tagged with the leaf counter too, so a granule left by an
// earlier leaf never passes for a current one (no clearing between leaves,
// whatever their participant counts).  Rows never move inside the
// leaf (logical pivoting); every wave replays the LAPACK interchange sequence
// in its lanes, which gives ipiv, the net row movement and, for the zero
// rule, the row on the diagonal.  Every spin is bounded (200 ms) and reports
// through info[1].
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "device_common.h"

namespace gelim {
namespace big {
namespace leafk {

constexpr int LW = 32;             // leaf width
constexpr int R = 4;               // rows per lane of the default shape (template parameter RW)
constexpr int kRowsPerWave = 64 * R;
constexpr int kMaxP = 256;         // participating workgroups
constexpr int kAuxSc1 = 16;        // buffer-op aux: sc1
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Exchange workspace: per (set, parity, participant) one key granule and
// the candidate row as LW data-tagged granules.
struct Xchg {
  u32x4* key;   // [2 sets][2 parities][kMaxP] {key lo, key hi, row, seq}
  u32x4* row;   // [2 sets][2 parities][kMaxP][LW] {value lo, value hi, row, seq}
};
constexpr size_t kKeyBytes = (size_t)2 * 2 * kMaxP * 16;
constexpr size_t kRowBytes = (size_t)2 * 2 * kMaxP * LW * 16;

struct LeafArgs {
  double* A;         // leaf top-left: row c0, column c0 of the system
  int64_t lda;
  int m;             // rows n - c0 (>= LW)
  int col0;          // c0 (absolute column / row of the leaf's diagonal)
  int P;             // participating workgroups
  int leaf;          // leaf counter of the solve: granule set = leaf & 1, and the tag of
                     // every granule of column J is (leaf << 6) | (J + 1) -- unique within a
                     // solve, so nothing stale can ever match (the driver zeroes the area
                     // before every solve)
  int* ipiv;         // ipiv[c0 + J] = absolute row swapped with row c0 + J
  int* pairs;        // [0] = count, then (dst, src) rows relative to c0
  int* info;         // [0] 1 + first zero-pivot column (kept if set), [1] hand-off error
  Xchg x;
  unsigned long long* stamps;  // diagnostics (null in production): [P][LW][8] shader clocks
};

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
__device__ __forceinline__ uint64_t u64of(unsigned lo, unsigned hi) { return ((uint64_t)hi << 32) | lo; }

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

// Diagnostic phase stamp of column J (lane 0 of wave 0 of every participant):
// 0 start, 1 arg-max done, 2 published + pending update applied, 3 key
// sweep ready, 4 pivot row loaded, 5 pivot row in LDS, 6 multipliers and
// next column done, 7 key sweeps + 256 * row loads
// (call sites test g.stamps first, so production runs issue no s_memtime: an
// SMEM op in flight would also hold every lgkmcnt(0) wait for the LDS)
__device__ __forceinline__ void lstamp(const LeafArgs& g, int J, int k, unsigned long long v) {
  if (g.stamps != nullptr && threadIdx.x == 0) g.stamps[((int64_t)blockIdx.x * LW + J) * 8 + k] = v;
}

template <int NWV, int RW>
struct alignas(16) LeafLds {
  double prow[NWV][2][LW];      // per wave: the pivot rows of the last two columns (parity)
  double cand[2][NWV][LW];      // per parity and wave: the wave's candidate row (NWV > 1)
  u32x4 wkey[2][NWV];           // per parity and wave: {key lo, key hi, row, -} (NWV > 1)
  int dest[NWV][64 * RW];       // final row of a moved local row (-1: unmoved)
};

// ---- the LAPACK interchange replay, in the lanes of the wave -----------------
// Lane e < cnt holds one displaced row: trow (row index, relative to c0) now
// at position tpos.  Rows not in the table sit at their own index.
struct Table {
  int trow, tpos, cnt;
};

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

// Wave arg-max of (key, row): largest key, lowest row; returns the winning
// lane (-1 when every key is 0).  DPP max of the high word + one ballot; the
// exact 64-bit / lowest-row resolution only on high-word ties.
__device__ __forceinline__ int wave_argmax_lane(uint64_t k, unsigned row) {
  const unsigned h = (unsigned)(k >> 32);
  const unsigned hm = dev::wave_max_u32(h);
  const bool c1 = h == hm && k != 0;
  const uint64_t hold = __ballot(c1);
  if (hold == 0) return -1;
  if (__popcll(hold) == 1) return __ffsll((long long)hold) - 1;
  const unsigned lm = dev::wave_max_u32(c1 ? (unsigned)k : 0u);
  const bool c2 = c1 && (unsigned)k == lm;
  const unsigned mr = dev::wave_min_u32(c2 ? row : 0xffffffffu);
  return __ffsll((long long)__ballot(c2 && row == mr)) - 1;
}

// First live column of a candidate row at column J: J - 1 (the row's own
// multiplier of the pending update) and everything right of it.
template <int J>
constexpr int kLive = J > 0 ? J - 1 : 0;

// Granule index g = participant * LW + column of a row sweep at column J,
// with dead columns redirected to the participant's first live one: the
// lanes then share that line and the sweep moves only the live bytes.
template <int J>
__device__ __forceinline__ int live_granule(int g) {
  return (g % LW) < kLive<J> ? g - (g % LW) + kLive<J> : g;
}

template <int MODE, int NKK, int NR, int NWV, int R = leafk::R>
struct Leaf {
  using Lds = LeafLds<NWV, R>;
  // one column J of the leaf (compile time); false: hand-off aborted
  template <int J>
  static __device__ __forceinline__ bool col(double (&a)[R][LW], bool (&live)[R], int (&pos)[R], double (&lp)[R],
                                             Lds& sh, Table& tb, const LeafArgs& g, int lane, int wave, int base) {
    constexpr int par = J & 1;
    lane = opq(lane);
    const int part = blockIdx.x;
    const unsigned seq = ((unsigned)g.leaf << 6) | (unsigned)(J + 1);
    const int slot = ((g.leaf & 1) * 2 + par) * kMaxP;
    double* prow = &sh.prow[wave][0][0];  // [2][LW], this wave's
    if (g.stamps != nullptr) lstamp(g, J, 0, __builtin_amdgcn_s_memtime());
    // 1. this lane's candidate: best live row (rows grow with the slot, so a
    //    strict '>' keeps the lowest row on ties)
    //    ZERO rule: the diagonal is the row at POSITION J and "the first
    //    non-zero row below" is the lowest POSITION, so the key is
    //    class<<32 | ~position (each lane tracks its rows' positions)
    uint64_t bk = 0;
    int bi = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      uint64_t k = dev::pivot_ukey_t<MODE>(a[i][J], pos[i] == J, live[i]);
      if constexpr (MODE == 0) k = k == 0 ? 0 : (k << 32) | (0xffffffffu - (unsigned)pos[i]);
      const bool c = k > bk;
      bk = c ? k : bk;
      bi = c ? i : bi;
    }
    const unsigned brow = (unsigned)(base + lane + 64 * bi);
    // 2. this wave's candidate
    const int wl = wave_argmax_lane(bk, brow);
    if (g.stamps != nullptr) lstamp(g, J, 1, __builtin_amdgcn_s_memtime());
    // the winner's row goes through LDS (the winning lane writes it, lane c
    // reads element c) so the LW granules leave in ONE 32-lane store instead
    // of LW single-lane ones.  The slot is wave-uniform (readlane): every
    // slot branch is a uniform one over compile-time indices, so the register
    // panel is never dynamically indexed.
    double* cand = &sh.cand[NWV > 1 ? par : 0][wave][0];
    if (wl >= 0) {
      const int wbi = __builtin_amdgcn_readlane(bi, wl);
#pragma unroll
      for (int i = 0; i < R; ++i)
        if (wbi == i && lane == wl) {
#pragma unroll
          for (int c = 0; c < LW; c += 2) {
            const double x = a[i][c], y = a[i][c + 1];
            asm volatile("" ::"v"(x), "v"(y));
            *reinterpret_cast<double2*>(&cand[c]) = make_double2(x, y);
          }
        }
    }
    // 3. publish the participant's candidate: LW data-tagged granules
    //    {value, row, seq}, then its key granule; no drain and no flag -- a
    //    reader trusts a granule exactly when its seq matches (16-byte sc1
    //    store / load, untorn on gfx950).  Only columns J-1.. of the
    //    candidate matter from column J on (J-1: the row's own multiplier of
    //    the pending update): dead granules are neither stored nor read
    {
      const __amdgpu_buffer_rsrc_t rk = rsrc(g.x.key + slot + part, 16);
      const __amdgpu_buffer_rsrc_t rr = rsrc(g.x.row + (int64_t)(slot + part) * LW, LW * 16);
      if constexpr (NWV == 1) {
        if (wl >= 0) {
          const unsigned wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, wl);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local LDS hand-off
          if (lane < LW && lane >= kLive<J>) {
            const double x = cand[lane];
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo32(x), hi32(x), wrow, seq}, rr, lane * 16, 0, kAuxSc1);
          }
          if (lane == wl)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)bk, (unsigned)(bk >> 32), brow, seq}, rk, 0, 0,
                                                   kAuxSc1);
        } else if (lane == 0) {  // no live row here: an empty candidate
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0xffffffffu, seq}, rk, 0, 0, kAuxSc1);
        }
      } else {
        // the waves' candidates merge in LDS behind one barrier; wave 0
        // publishes the winner.  Parity buffers: a wave writes parity J+1
        // only after column J's exchange completed, which needs this
        // participant's column-J publish, which follows every wave's arrival
        // at this barrier -- so no wave still reads parity J&1 data of J-2.
        if (wl >= 0) {
          if (lane == wl) sh.wkey[par][wave] = u32x4{(unsigned)bk, (unsigned)(bk >> 32), brow, 0u};
        } else if (lane == 0) {
          sh.wkey[par][wave] = u32x4{0u, 0u, 0xffffffffu, 0u};
        }
        __syncthreads();
        if (wave == 0) {
          u32x4 kb = sh.wkey[par][0];
          int wv = 0;
#pragma unroll
          for (int w = 1; w < NWV; ++w) {
            const u32x4 kk = sh.wkey[par][w];
            const uint64_t k1 = u64of(kk.x, kk.y), k0 = u64of(kb.x, kb.y);
            const bool c = k1 > k0 || (k1 == k0 && k1 != 0 && kk.z < kb.z);
            kb = c ? kk : kb;
            wv = c ? w : wv;
          }
          if (u64of(kb.x, kb.y) != 0) {
            if (lane < LW && lane >= kLive<J>) {
              const double x = sh.cand[par][wv][lane];
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo32(x), hi32(x), kb.z, seq}, rr, lane * 16, 0, kAuxSc1);
            }
            if (lane == 63) __builtin_amdgcn_raw_buffer_store_b128(u32x4{kb.x, kb.y, kb.z, seq}, rk, 0, 0, kAuxSc1);
          } else if (lane == 0) {
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{0u, 0u, 0xffffffffu, seq}, rk, 0, 0, kAuxSc1);
          }
        }
      }
    }
    // 3b. while the exchange is in flight: the previous pivot's rank-1
    //     update of columns J+1.. (column J got it already, it is the one
    //     the candidate above was computed on)
    if constexpr (J > 0) {
#pragma unroll
      for (int c = J + 1; c < LW; ++c) {
        const double uc = prow[((J - 1) & 1) * LW + c];
#pragma unroll
        for (int i = 0; i < R; ++i) a[i][c] = fma(-lp[i], uc, a[i][c]);
      }
    }
    if (g.stamps != nullptr) lstamp(g, J, 2, __builtin_amdgcn_s_memtime());
    // 4. sweep: lane p (+ 64 k) reads participant p's key and, when the
    //    candidate rows fit (NR > 0), every participant's row too -- granule
    //    p*LW + c sits in load p/2 of lane 32 (p&1) + c -- so the winner's
    //    row normally arrives with the last key sweep (one round trip per
    //    column instead of two).  All loads unconditional and in flight at
    //    once (clamped: a predicated load is a branch with its own vmcnt(0)).
    const __amdgpu_buffer_rsrc_t rks = rsrc(g.x.key + slot, kMaxP * 16);
    const __amdgpu_buffer_rsrc_t rrw = rsrc(g.x.row + (int64_t)slot * LW, kMaxP * LW * 16);
    u32x4 kv[NKK];
    u32x4 rw[NR > 0 ? NR : 1];
    unsigned long long t0 = 0;
    int sweeps = 0;
    for (int it = 0;; ++it) {
#pragma unroll
      for (int k = 0; k < NKK; ++k)
        kv[k] = __builtin_amdgcn_raw_buffer_load_b128(rks, min(k * 64 + lane, g.P - 1) * 16, 0, kAuxSc1);
      if constexpr (NR > 0) {
#pragma unroll
        for (int k = 0; k < NR; ++k)
          rw[k] = __builtin_amdgcn_raw_buffer_load_b128(rrw, min(live_granule<J>(k * 64 + lane), g.P * LW - 1) * 16, 0,
                                                        kAuxSc1);
      }
      bool ready = true;
#pragma unroll
      for (int k = 0; k < NKK; ++k) ready = ready && kv[k].w == seq;
      if (__ballot(!ready) == 0) {
        sweeps = it + 1;
        break;
      }
      if ((it & 63) == 63) {  // abort / timeout checks every 64 sweeps (each is a round trip)
        if (t0 == 0) t0 = rtc();
        else if (rtc() - t0 > kSpinTicks) {
          __hip_atomic_store(g.info + 1, 5, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return false;
        }
        if (__hip_atomic_load(g.info + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return false;
      }
    }
    if (g.stamps != nullptr) lstamp(g, J, 3, __builtin_amdgcn_s_memtime());
    // 5. global winner (largest key, lowest row); lanes past P hold clamped
    //    duplicates, which never change the arg-max
    uint64_t key = u64of(kv[0].x, kv[0].y);
    unsigned krow = kv[0].z;
    int kp = lane;
#pragma unroll
    for (int k = 1; k < NKK; ++k) {
      const uint64_t kk = u64of(kv[k].x, kv[k].y);
      const bool c = kk > key || (kk == key && kk != 0 && kv[k].z < krow);
      key = c ? kk : key;
      krow = c ? kv[k].z : krow;
      kp = c ? min(k * 64 + lane, g.P - 1) : kp;
    }
    kp = min(kp, g.P - 1);
    const int wlw = wave_argmax_lane(key, krow);
    const int pw = __builtin_amdgcn_readlane(kp, wlw);
    const unsigned pr = (unsigned)__builtin_amdgcn_readlane((int)krow, wlw);
    // 6. the winner's row in the lanes of half h = pw & 1 (lane 32 h + c
    //    holds column c): from the sweep when it carried the rows, re-read
    //    until every granule is current (the row was stored before the key,
    //    but nothing orders them)
    const int h = pw & 1;
    const bool mine = (lane >> 5) == h;
    const __amdgpu_buffer_rsrc_t rrs = rsrc(g.x.row + (int64_t)(slot + pw) * LW, LW * 16);
    u32x4 rv;
    if constexpr (NR > 0) {
      rv = rw[0];
#pragma unroll
      for (int k = 1; k < NR; ++k) rv = (k == (pw >> 1)) ? rw[k] : rv;
    } else {
      rv = __builtin_amdgcn_raw_buffer_load_b128(rrs, max(lane & (LW - 1), kLive<J>) * 16, 0, kAuxSc1);
    }
    int rl = 0;
    while (__ballot(mine && (lane & (LW - 1)) >= kLive<J> && rv.w != seq) != 0) {
      rv = __builtin_amdgcn_raw_buffer_load_b128(rrs, max(lane & (LW - 1), kLive<J>) * 16, 0, kAuxSc1);
      if ((++rl & 63) == 63 && __hip_atomic_load(g.info + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
        return false;
    }
    if (g.stamps != nullptr) lstamp(g, J, 4, __builtin_amdgcn_s_memtime());
    // the winner published its row before applying the pending update of
    // pivot J-1 to columns J+1..: apply it here, with the row's own
    // multiplier (its column J-1) -- the very FMA its owner performs
    const int cc = lane & (LW - 1);
    double pval = mkd(rv.x, rv.y);
    if constexpr (J > 0) {
      const double lw = mkd((unsigned)__builtin_amdgcn_readlane((int)rv.x, 32 * h + J - 1),
                            (unsigned)__builtin_amdgcn_readlane((int)rv.y, 32 * h + J - 1));
      if (mine && cc > J) pval = fma(-lw, prow[((J - 1) & 1) * LW + cc], pval);
    }
    if (mine) prow[par * LW + cc] = pval;
    // interchange replay; participant 0 records the LAPACK pivot
    const int qpos = table_swap(tb, J, (int)pr, lane);
    if constexpr (MODE == 0) {  // positions J and qpos exchange their rows
#pragma unroll
      for (int i = 0; i < R; ++i)
        pos[i] = (base + lane + 64 * i == (int)pr) ? J : (pos[i] == J ? qpos : pos[i]);
    }
    if (part == 0 && wave == 0 && lane == 0) g.ipiv[g.col0 + J] = g.col0 + qpos;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the pivot row is in LDS (wave-local)
    if (g.stamps != nullptr) lstamp(g, J, 5, __builtin_amdgcn_s_memtime());
    lstamp(g, J, 7, (unsigned long long)sweeps + 256ull * rl);

    // 7. multipliers; this pivot's update of column J+1 only (the next
    //    candidate), the rest of it is pending until the next exchange
    const double pv = prow[par * LW + J];
    const bool zero = !(pv != 0.0);
    const double rinv = zero ? 0.0 : recip(pv);
    if (zero && part == 0 && wave == 0 && lane == 0 && g.info[0] == 0) atomicCAS(g.info, 0, g.col0 + J + 1);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      live[i] = live[i] && (base + lane + 64 * i != (int)pr);
      lp[i] = live[i] ? a[i][J] * rinv : 0.0;
      a[i][J] = live[i] ? lp[i] : a[i][J];
    }
    if constexpr (J + 1 < LW) {
      const double uc = prow[par * LW + J + 1];
#pragma unroll
      for (int i = 0; i < R; ++i) a[i][J + 1] = fma(-lp[i], uc, a[i][J + 1]);
    }
    if (g.stamps != nullptr) {
      asm volatile("" ::"v"(a[R - 1][LW - 1]));
      if (g.stamps != nullptr) lstamp(g, J, 6, __builtin_amdgcn_s_memtime());
    }
    return true;
  }

  template <int... J>
  static __device__ __forceinline__ bool factor(double (&a)[R][LW], bool (&live)[R], int (&pos)[R], Lds& sh,
                                                Table& tb, const LeafArgs& g, int lane, int wave, int base,
                                                std::integer_sequence<int, J...>) {
    double lp[R];  // multipliers of the pending (previous) pivot
#pragma unroll
    for (int i = 0; i < R; ++i) lp[i] = 0.0;
    return (col<J>(a, live, pos, lp, sh, tb, g, lane, wave, base) && ...);
  }
};

template <int MODE, int NKK, int NR, int NWV, int R>
__global__ __launch_bounds__(64 * NWV, 1) void leaf_kernel(LeafArgs g) {
  constexpr int kRowsPerWave = 64 * R;
  __shared__ LeafLds<NWV, R> sh;
  const int lane = threadIdx.x & 63;
  const int wave = NWV > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  const int base = (blockIdx.x * NWV + wave) * kRowsPerWave;
  double a[R][LW];
  bool live[R];
  int pos[R];  // ZERO rule: current position of each row (unused for PARTIAL)
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = base + lane + 64 * i;
    live[i] = r < g.m;
    pos[i] = r;
    const double2* src = reinterpret_cast<const double2*>(g.A + (int64_t)min(r, g.m - 1) * g.lda);
#pragma unroll
    for (int c = 0; c < LW; c += 2) {
      const double2 x = src[c / 2];
      a[i][c] = x.x;
      a[i][c + 1] = x.y;
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) sh.dest[wave][lane + 64 * i] = -1;
  Table tb{0, 0, 0};
  if (!Leaf<MODE, NKK, NR, NWV, R>::factor(a, live, pos, sh, tb, g, lane, wave, base,
                                        std::make_integer_sequence<int, LW>{}))
    return;

  // net row movement (participant 0 publishes it); every wave maps its own
  // moved rows to their final positions and writes its rows there
  if (blockIdx.x == 0 && wave == 0) {
    if (lane < tb.cnt) {
      g.pairs[1 + 2 * lane] = tb.tpos;
      g.pairs[2 + 2 * lane] = tb.trow;
    }
    if (lane == 0) g.pairs[0] = tb.cnt;
  }
  if (lane < tb.cnt && tb.trow >= base && tb.trow < base + kRowsPerWave) sh.dest[wave][tb.trow - base] = tb.tpos;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = base + lane + 64 * i;
    if (r < g.m) {
      const int d = sh.dest[wave][lane + 64 * i];
      double2* dst = reinterpret_cast<double2*>(g.A + (int64_t)(d < 0 ? r : d) * g.lda);
#pragma unroll
      for (int c = 0; c < LW; c += 2) dst[c / 2] = make_double2(a[i][c], a[i][c + 1]);
    }
  }
}

// launcher of one instantiation (leaf_w*.hip): NWV waves of RW rows per
// lane per participant
template <int MODE, int NKK, int NR, int NWV, int RW>
void launch_leaf(const LeafArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((leaf_kernel<MODE, NKK, NR, NWV, RW>), dim3((unsigned)a.P), dim3(64 * NWV), 0, s, a);
}

// host dispatch by participant count, one (NWV, RW, MODE) per instantiation unit
template <int NWV, int RW, int MODE>
void launch_leaf_shape(const LeafArgs& a, bool fused, hipStream_t s);

#define GELIM_LEAF_SHAPE_DEFINE(NWV, RW, MODE)                                                  \
  template <>                                                                                   \
  void launch_leaf_shape<NWV, RW, MODE>(const LeafArgs& a, bool fused, hipStream_t s) {         \
    if (fused && a.P <= 8) launch_leaf<MODE, 1, 4, NWV, RW>(a, s);                              \
    else if (fused && a.P <= 16) launch_leaf<MODE, 1, 8, NWV, RW>(a, s);                        \
    else if (fused && a.P <= 32) launch_leaf<MODE, 1, 16, NWV, RW>(a, s);                       \
    else if (a.P <= 64) launch_leaf<MODE, 1, 0, NWV, RW>(a, s);                                 \
    else if (a.P <= 128) launch_leaf<MODE, 2, 0, NWV, RW>(a, s);                                \
    else launch_leaf<MODE, 4, 0, NWV, RW>(a, s);                                                \
  }

}  // namespace leafk
}  // namespace big
}  // namespace gelim
