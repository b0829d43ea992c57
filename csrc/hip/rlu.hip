// Resident LU ("rlu"): the whole blocked LU with partial pivoting of an
// n <= 2048 augmented system [A | b] in ONE persistent launch, with the
// matrix resident in registers for the whole factorisation.
//
// What it computes: the reference's forward elimination (getPivot +
// computeGauss, OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:123-182,
// partial pivoting; the internal programs' zero-pivot rule as MODE 0,
// Pthreads/Version-1/gauss_internal_input.c:75-121) as a right-looking
// blocked LU: U rows and the transformed b (y) end up in `work` at their
// physical row positions, the pivot row of every column in `piv`; back
// substitution (backsub.hip, row indirection through piv) follows.
//
// How (MI355X-first; the fused step schedule of lu_panel.hip re-read and
// re-wrote its 256 KB panel through one CU every step and paid a launch
// boundary plus a narrow-update kernel per step):
//  * logical pivoting for the WHOLE factorisation: rows never move.  Thread
//    t of every workgroup owns the physical rows t, t+512, t+1024, ... (R
//    slots), so a row always sits in the same lane of every workgroup and no
//    row interchange ever crosses lanes or workgroups;
//  * workgroup 0 (the "engine") keeps the current 16-column panel in VGPRs
//    across ALL steps: it factors panel j (one barrier per column), then
//    applies step j to panel j+1's strip itself and goes straight on -- the
//    next panel is never written back;
//  * workgroups 1..np (the "updaters") each keep one 16-column strip (the
//    last one: b) in VGPRs and apply every published step to it on their own
//    CU: per step they read the 16 pivot rows' L11, do the 16x16 TRSM with a
//    DPP row broadcast, and a rank-16 VALU update whose U12 operands come
//    from the scalar cache (s_load -> SGPR operands: no LDS or VALU traffic
//    for the broadcast).  fp64 VALU and fp64 MFMA have the same rate on
//    CDNA4 (78.6 TF each), so the register layout decides, not the matrix
//    core;
//  * hand-offs follow the write-through recipe (cdna_hip_programming.md §6
//    Guideline 16, R1): payload stored sc1, every storing wave drains,
//    barrier, one lane stores the flag; consumers poll one word relaxed and
//    read the payload with sc1 loads only.  Every spin is bounded (200 ms of
//    s_memrealtime) and sets an error word, so the grid always drains;
//  * U rows go straight to `work` at the step their row is retired.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace rlu {
namespace {

// Threads per workgroup NT (a template parameter): 512 = 8 wave64s, 2 per
// SIMD (R <= 4 row slots), or 1024 = 16 wave64s (R <= 2: the n <= 2048
// engine on the 2-slot register budget, 128 VGPRs, where 512 threads need 4
// slots and spill).
constexpr int kWavesMax = 16;
constexpr int kW = 16;           // panel / strip width
constexpr int kAuxSc1 = 16;      // buffer-op aux: sc1 (write-through store, L1-bypass load)
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x8 __attribute__((ext_vector_type(8)));

struct Args {
  const double* src;  // input augmented system, n x (n+1), leading dim lds
  int64_t lds;
  double* work;       // output: U rows at their physical positions, y in column n
  int64_t ldw;
  int n, np;          // order, number of 16-column panels
  int* piv;           // [n] physical row of the pivot of every column
  int* info;          // [0]: 1 + first zero-pivot column; [1]: hand-off timeout code
  unsigned* flags;    // [np] L published, [np + 1] strip published (zeroed per launch)
  double* lbuf;       // [np][R*8][NT] double2: each panel's multipliers, thread-major
  double* pbuf;       // [np][16][16]: each panel's pivot rows (L11 | U11)
  double* ubuf;       // [np][np + 1][16][16]: U12 of (step, strip), column-major
  double* hbuf;       // [np + 1][R*8][NT] double2: strips handed to the engine
  int* pslot;         // [np][32]: each panel's 16 pivot rows on a 128-byte line of its own
  int pslot_mode;     // 1: updaters read the pivots from pslot, 0: from piv
  unsigned long long* stamps;  // diagnostics (null in production): realtime per phase
};

struct alignas(16) Shared {
  double cand[2][kWavesMax][18];  // each wave's winning row (16 values) + 1/pivot
  u32x4 ckey[2][kWavesMax];       // {key hi, key lo, row, -}
  double prow[kW][kW];         // this panel's pivot rows (engine) / L11 (updaters)
  double xs[kW][kW];           // TRSM right-hand sides (updaters)
  int sel[kW];                 // physical pivot row of each panel column
  unsigned fb[kWavesMax];         // singular fallback: lowest live row per wave
  int ok[2];                   // poll results (parity-buffered)
};

// ---- small device helpers ------------------------------------------------

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ unsigned long long cyc() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// Diagnostic phase stamps (s_memrealtime, 10 ns ticks), written by thread 0.
__device__ __forceinline__ void stamp(const Args& g, int idx) {
  if (g.stamps != nullptr && threadIdx.x == 0) g.stamps[idx] = rtc();
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ unsigned lo32(double x) { return (unsigned)__double_as_longlong(x); }
__device__ __forceinline__ unsigned hi32(double x) {
  return (unsigned)((uint64_t)__double_as_longlong(x) >> 32);
}
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Value barrier: the compiler must treat x as freshly defined here, so
// expressions of lane indices are recomputed inside the step loop instead of
// being hoisted out of it (hoisted per-column LDS addresses and compare masks
// cost ~60 VGPRs/SGPRs and spill the panel).
template <typename T>
__device__ __forceinline__ T opq(T x) {
  asm volatile("" : "+v"(x));
  return x;
}

// Thread-major panel buffers: groups of 4 consecutive threads own one
// contiguous block of R*8*64 bytes, laid out [slot][pair][thread%4] in
// 16-byte pieces.  The per-thread part is ONE voffset VGPR (tvo), the
// (slot, pair) part a small constant the assembler folds into the
// instruction's 12-bit immediate offset -- no per-(slot, pair) SGPRs or
// VGPRs, which LICM would otherwise pin for the whole factorisation.  A wave
// access touches 16 contiguous 64-byte segments.
template <int R>
__device__ __forceinline__ constexpr int tvo(int t) { return (t >> 2) * (R * 512) + (t & 3) * 16; }
__device__ __forceinline__ constexpr int soff(int i, int cp) { return (i * 8 + cp) * 64; }

__device__ __forceinline__ void st128(__amdgpu_buffer_rsrc_t r, int voff, int so, double x, double y) {
  const u32x4 v = {lo32(x), hi32(x), lo32(y), hi32(y)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, so, kAuxSc1);
}

__device__ __forceinline__ void st64(__amdgpu_buffer_rsrc_t r, int voff, double x) {
  const u32x2 v = {lo32(x), hi32(x)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, voff, 0, kAuxSc1);
}

__device__ __forceinline__ void st32(__amdgpu_buffer_rsrc_t r, int voff, int x) {
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)x, r, voff, 0, kAuxSc1);
}

__device__ __forceinline__ u32x4 ld128(__amdgpu_buffer_rsrc_t r, int voff, int so) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, voff, so, kAuxSc1);
}

__device__ __forceinline__ double ld64(__amdgpu_buffer_rsrc_t r, int voff) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, kAuxSc1);
  return mkd(v.x, v.y);
}

__device__ __forceinline__ int ld32(__amdgpu_buffer_rsrc_t r, int voff) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, kAuxSc1);
}

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void set_flag(unsigned* f) {
  __hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Whole workgroup: wait until *f != 0 (thread 0 polls relaxed, with s_sleep);
// false when the bounded spin ran out or another workgroup already gave up.
__device__ __forceinline__ bool wait_flag(unsigned* f, int* err, Shared& sh, int par, int code) {
  if (threadIdx.x == 0) {
    int ok = 1;
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      const unsigned long long t0 = rtc();
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          ok = 0;
          break;
        }
        if (rtc() - t0 > kSpinTicks) {
          __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    sh.ok[par] = ok;
  }
  __syncthreads();
  return sh.ok[par] != 0;
}

template <int CTRL>
__device__ __forceinline__ unsigned dpp(unsigned identity, unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, 0xf, 0xf, false);
}

// Forward-substitution step I of the 16x16 unit-lower TRSM: lane J of a
// 16-lane DPP row holds x[J] of one column; x[I] is broadcast to the row
// with row_newbcast:I (no LDS round trip on the 16-step chain).
template <int I>
__device__ __forceinline__ void trsm_step(double& x, const double (&lrow)[kW], int j) {
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)hi32(x), 0x150 + I, 0xf, 0xf, false);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)lo32(x), 0x150 + I, 0xf, 0xf, false);
  x = (j > I) ? fma(-lrow[I], mkd(lo, hi), x) : x;
}

template <int... I>
__device__ __forceinline__ void trsm(double& x, const double (&lrow)[kW], int j,
                                     std::integer_sequence<int, I...>) {
  j = opq(j);
  (trsm_step<I>(x, lrow, j), ...);
}

// U12 (ut: column-major 16x16) reaches the FMAs as SGPR operands through
// the scalar cache: one column = two 64-byte loads and ONE wait.  `dep` (the
// previous column's result) keeps the scheduler from hoisting all columns'
// loads to the top, where their 512 SGPRs would spill; a hand-pipelined
// issue/wait pair is not safe (the register allocator may copy a still
// pending destination).
template <int OFF>
__device__ __forceinline__ void sload16(const double* p, double dep, f64x8& lo, f64x8& hi) {
  asm volatile(
      "s_load_dwordx16 %0, %2, %3\n\t"
      "s_load_dwordx16 %1, %2, %4\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(lo), "=&s"(hi)
      : "s"(p), "n"(OFF), "n"(OFF + 64), "v"(dep)
      : "memory");
}

template <int C>
__device__ __forceinline__ void rank16_col(double (&s)[kW], const double (&L)[kW], const double* ut, int ws) {
  if (C < ws) {  // uniform (narrow strips: the b column)
    f64x8 u0, u1;
    sload16<C * 128>(ut, s[C > 0 ? C - 1 : 0], u0, u1);
    double a0 = s[C], a1 = 0.0;
#pragma unroll
    for (int I = 0; I < 8; ++I) {
      a0 = fma(-L[I], u0[I], a0);
      a1 = fma(-L[8 + I], u1[I], a1);
    }
    s[C] = a0 + a1;
  }
}

template <int... C>
__device__ __forceinline__ void rank16_c(double (&s)[kW], const double (&L)[kW], const double* ut, int ws,
                                         std::integer_sequence<int, C...>) {
  (rank16_col<C>(s, L, ut, ws), ...);
}

// Pull U12's 32 lines into the scalar cache in parallel (4 per wave), so
// the per-slot column loads of every wave hit.
__device__ __forceinline__ void warm_u12(const double* ut) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) & 7;
  const double* p = ut + 8 * w;  // line w; lines w + 8k are 512 bytes apart
  f64x8 a, b;
  asm volatile(
      "s_load_dwordx16 %0, %2, 0x0\n\t"
      "s_load_dwordx16 %1, %2, 0x200\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_load_dwordx16 %0, %2, 0x400\n\t"
      "s_load_dwordx16 %1, %2, 0x600\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&s"(a), "=&s"(b)
      : "s"(p)
      : "memory");
}

__device__ __forceinline__ void rank16(double (&s)[kW], const double (&L)[kW], const double* ut, int ws) {
  rank16_c(s, L, ut, ws, std::make_integer_sequence<int, kW>{});
}

// Store one register row to LDS from inside a per-slot branch.  The empty
// asm keeps every branch's values distinct: without it LLVM merges the slot
// branches into one store through a phi of row POINTERS, which demotes the
// whole register panel to scratch memory.
__device__ __forceinline__ void put_row(double2* dst, const double (&row)[kW]) {
#pragma unroll
  for (int cp = 0; cp < 8; ++cp) {
    const double x = row[2 * cp], y = row[2 * cp + 1];
    asm volatile("" ::"v"(x), "v"(y));
    dst[cp] = make_double2(x, y);
  }
}

// Compile-time loop: f(std::integral_constant<int, I>) for I = 0..N-1, so
// register arrays indexed by I never become dynamically indexed (a rolled
// slot loop demotes the whole panel to scratch memory).
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// 1/p from v_rcp_f64 plus two Newton steps (3 dependent VALU pairs instead of
// the ~10-instruction IEEE division; multipliers within an ulp of a/p).
__device__ __forceinline__ double recip(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  return fma(r, fma(-p, r, 1.0), r);
}

// ---- the engine: panel factorisation in registers ------------------------

template <int NT, int R, int MODE>
struct Engine {
  static constexpr int kWaves = NT / 64;
  // One column J (compile time) of the panel whose first column is k0.
  template <int J>
  static __device__ __forceinline__ void col(double (&a)[R][kW], bool (&live)[R], int (&pos)[R], Shared& sh,
                                             int t, int lane, int wave, int w, int k0, int* info,
                                             unsigned long long* cs, unsigned* pend) {
    if (J >= w) return;  // uniform
    // diagnostics: shader-clock stamps of column 4 (cs != null only when stamping)
    auto mark = [&](int k) {
      if constexpr (J == 4) {
        if (cs != nullptr) {
          const unsigned long long v = cyc();
          if (t == 0) cs[k] = v;
        }
      }
    };
    mark(0);
    constexpr int par = J & 1;
    t = opq(t);
    lane = opq(lane);
    wave = opq(wave);

    // 1. this lane's candidate over its live rows (rows increase with the
    //    slot: strict '>' keeps the lowest row on ties, like getPivot).
    //    Bitwise '&' on the predicates: no short-circuit branches.
    double bv = 0.0;
    int bs = R;
    unsigned h = 0;
    if constexpr (MODE == 1) {
      // pairwise tree over the slots (depth log2 R instead of a serial
      // chain); a dead or zero slot never wins, the lower slot wins ties
      double v[R];
      int sl[R];
#pragma unroll
      for (int i = 0; i < R; ++i) {
        v[i] = live[i] ? a[i][J] : 0.0;
        sl[i] = live[i] ? i : R;
      }
#pragma unroll
      for (int st = 1; st < R; st <<= 1)
#pragma unroll
        for (int i = 0; i + st < R; i += 2 * st) {
          const bool c = fabs(v[i + st]) > fabs(v[i]);
          v[i] = c ? v[i + st] : v[i];
          sl[i] = c ? sl[i + st] : sl[i];
        }
      bv = v[0];
      bs = (bv != 0.0) ? sl[0] : R;
      h = (hi32(bv) & 0x7fffffffu) + (bs < R ? 1u : 0u);
    } else {
      // ZERO rule (Pthreads/Version-1/gauss_internal_input.c:75-121): the row
      // at POSITION k0+J (after every earlier interchange) is "the diagonal"
      // when non-zero, else the live non-zero row at the lowest position:
      // key = class<<30 | ~position.  Rows never move here, so each lane
      // tracks the current position of its rows (pos[], updated per pivot)
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double v = a[i][J];
        const bool nz = live[i] & (v == v) & (v != 0.0);
        const unsigned key = nz ? ((((pos[i] == k0 + J) ? 2u : 1u) << 30) | (0x3fffffffu - (unsigned)pos[i])) : 0u;
        const bool c = key > h;
        h = c ? key : h;
        bv = c ? v : bv;
        bs = c ? i : bs;
      }
    }
    // speculative, hidden under the arg-max: the value barrier keeps LLVM from
    // sinking the reciprocal into the winner's publish branch after the ladder
    const double rv = opq(recip(bv));
    mark(1);

    // 2. wave arg-max: DPP max of the 32-bit key and one ballot; the exact
    //    64-bit key + lowest-row resolution runs only on high-word ties
    const unsigned hmax = dev::wave_max_u32(h);
    unsigned wlo = 0, wrow = 0xffffffffu;
    if (hmax != 0) {
      int wl;
      const uint64_t hold = __ballot(h == hmax);
      if (MODE == 0 || __popcll(hold) == 1) {
        wl = __ffsll((long long)hold) - 1;
      } else {
        const unsigned lo = lo32(bv);
        const unsigned lomax = dev::wave_max_u32(h == hmax ? lo : 0u);
        const bool c2 = (h == hmax) & (lo == lomax);
        const uint64_t h2 = __ballot(c2);
        if (__popcll(h2) == 1) {
          wl = __ffsll((long long)h2) - 1;
        } else {
          const unsigned rowv = (unsigned)(t + bs * NT);
          const unsigned minrow = dev::wave_min_u32(c2 ? rowv : 0xffffffffu);
          wl = __ffsll((long long)__ballot(c2 & (rowv == minrow))) - 1;
        }
      }
      const int wbs = __builtin_amdgcn_readlane(bs, wl);
      wrow = (unsigned)(wave * 64 + wl + wbs * NT);
      if constexpr (MODE == 1) wlo = (unsigned)__builtin_amdgcn_readlane((int)lo32(bv), wl);
      // the wave's winner publishes its whole row (L11 part + U part) and 1/pivot
#pragma unroll
      for (int i = 0; i < R; ++i)
        if (wbs == i && lane == wl) {
          double2* dst = reinterpret_cast<double2*>(&sh.cand[par][wave][0]);
          put_row(dst, a[i]);
          dst[8] = make_double2(rv, 0.0);
        }
    }
    if (lane == 0) sh.ckey[par][wave] = u32x4{hmax, wlo, wrow, 0u};
    mark(2);
    // the previous step's multiplier stores (issued > 1 us ago) drain here,
    // behind this column's barrier, instead of on the engine's path between
    // steps; its flag follows the barrier
    if constexpr (J == 1) {
      if (pend != nullptr) drain();
    }
    __syncthreads();
    if constexpr (J == 1) {
      if (pend != nullptr && t == 0) set_flag(pend);
    }
    mark(3);

    // 3. merge the waves' candidates (lanes 0..7): max high key, exact on ties
    const u32x4 kk = sh.ckey[par][lane & (kWaves - 1)];
    unsigned gm = kk.x;
    gm = max(gm, dpp<0x111>(0u, gm));
    gm = max(gm, dpp<0x112>(0u, gm));
    gm = max(gm, dpp<0x114>(0u, gm));
    if constexpr (kWaves > 8) gm = max(gm, dpp<0x118>(0u, gm));
    const unsigned gh = (unsigned)__builtin_amdgcn_readlane((int)gm, kWaves - 1);
    int q = 0;
    unsigned p = 0;
    if (gh != 0) {
      const bool in = (lane < kWaves) & (kk.x == gh);
      const uint64_t hb = __ballot(in);
      if (__popcll(hb) == 1) {
        q = __ffsll((long long)hb) - 1;
      } else {
        const unsigned glo = dev::wave_max_u32(in ? kk.y : 0u);
        const bool in2 = in & (kk.y == glo);
        const unsigned mr = dev::wave_min_u32(in2 ? kk.z : 0xffffffffu);
        q = __ffsll((long long)__ballot(in2 & (kk.z == mr))) - 1;
      }
      p = (unsigned)__builtin_amdgcn_readlane((int)kk.z, q);
    } else {
      // singular column: no live row has a usable entry.  Record it, retire
      // the lowest live row with zero multipliers (the reference would stop).
      if (t == 0 && info[0] == 0) info[0] = k0 + J + 1;
      unsigned lr = 0xffffffffu;
#pragma unroll
      for (int i = R - 1; i >= 0; --i)  // ZERO: the row at the diagonal position (no interchange)
        lr = (live[i] && (MODE == 1 || pos[i] == k0 + J)) ? (unsigned)(t + i * NT) : lr;
      lr = dev::wave_min_u32(lr);
      if (lane == 0) sh.fb[wave] = lr;
      __syncthreads();
      p = 0xffffffffu;
#pragma unroll
      for (int v = 0; v < kWaves; ++v) p = min(p, sh.fb[v]);
      if (t == (int)(p % NT)) {
#pragma unroll
        for (int i = 0; i < R; ++i)
          if ((int)(p / NT) == i) {
            double2* dst = reinterpret_cast<double2*>(&sh.cand[par][0][0]);
            put_row(dst, a[i]);
            dst[8] = make_double2(0.0, 0.0);  // zero multipliers
          }
      }
      __syncthreads();
      q = 0;
    }

    mark(4);
    // 4. pivot row (uniform LDS reads), bookkeeping, multipliers, update
    //    (column J+1 first: the next column's search depends only on it)
    const double2* cr = reinterpret_cast<const double2*>(&sh.cand[par][q][0]);
    const double rinv = cr[8].x;
    double u[kW];
#pragma unroll
    for (int cp = (J + 1) / 2; cp < 8; ++cp) {
      const double2 v = cr[cp];
      u[2 * cp] = v.x;
      u[2 * cp + 1] = v.y;
    }
    if (wave == 0 && lane < 8) reinterpret_cast<double2*>(&sh.prow[J][0])[lane] = cr[lane];
    if (t == 0) sh.sel[J] = (int)p;
#pragma unroll
    for (int i = 0; i < R; ++i) live[i] = live[i] & (t + i * NT != (int)p);
    if constexpr (MODE == 0) {
      // interchange of positions k0+J and pos(p): p moves up to k0+J, the row
      // that sat there moves down to p's old position (read from its key)
      const int posp = gh != 0 ? (int)(0x3fffffffu - (gh & 0x3fffffffu)) : k0 + J;
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const bool isp = t + i * NT == (int)p;
        pos[i] = isp ? k0 + J : (pos[i] == k0 + J ? posp : pos[i]);
      }
    }
    double l[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      l[i] = a[i][J] * rinv;
      a[i][J] = l[i];
    }
    if constexpr (J + 1 < kW) {
#pragma unroll
      for (int i = 0; i < R; ++i) a[i][J + 1] = fma(-l[i], u[J + 1], a[i][J + 1]);
    }
    mark(5);
#pragma unroll
    for (int c = J + 2; c < kW; ++c)
#pragma unroll
      for (int i = 0; i < R; ++i) a[i][c] = fma(-l[i], u[c], a[i][c]);
    if constexpr (J == 4) asm volatile("" ::"v"(a[R - 1][kW - 1]));
    mark(6);
  }

  template <int... J>
  static __device__ __forceinline__ void factor(double (&a)[R][kW], bool (&live)[R], int (&pos)[R], Shared& sh,
                                                int t, int lane, int wave, int w, int k0, int* info,
                                                unsigned long long* cs, unsigned* pend,
                                                std::integer_sequence<int, J...>) {
    (col<J>(a, live, pos, sh, t, lane, wave, w, k0, info, cs, pend), ...);
  }
};

template <int NT, int R, int MODE>
__device__ __forceinline__ void engine(const Args& g, Shared& sh) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int vo = tvo<R>(t);  // this thread's voffset in the thread-major buffers
  const int n = g.n, np = g.np;
  constexpr int kPanelBytes = R * 8 * NT * 16;
  double a[R][kW];
  bool live[R];
  int pos[R];  // ZERO rule: current position of each row (unused for PARTIAL)
  // panel 0 straight from the input (8-byte loads: input rows need not be
  // 16-byte aligned); rows >= n read row n-1 and are never live
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int r = t + i * NT;
    live[i] = r < n;
    pos[i] = r;
    const double* rp = g.src + (int64_t)min(r, n - 1) * g.lds;
#pragma unroll
    for (int c = 0; c < kW; ++c) a[i][c] = rp[min(c, n - 1)];
  }
  const __amdgpu_buffer_rsrc_t rpiv = rsrc(g.piv, (uint32_t)n * 4);
  const __amdgpu_buffer_rsrc_t rps = rsrc(g.pslot, (uint32_t)np * 128);
  unsigned* pend = nullptr;  // the previous step's flag, set inside this step's column 1
  for (int j = 0; j < np; ++j) {
    const int k0 = kW * j;
    const int w = min(kW, n - k0);
    const bool more = j + 1 < np;
    stamp(g, j * 8 + 0);
    // the flag of the strip needed after this panel: its load is issued now
    // and its latency hides under the factorisation
    unsigned pre = 1;
    if (more && t == 0) pre = __hip_atomic_load(&g.flags[np + j + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long* cs = (g.stamps != nullptr && j == 10) ? g.stamps + 8 * np + 2 * (np + 1) * np : nullptr;
    Engine<NT, R, MODE>::factor(a, live, pos, sh, t, lane, wave, w, k0, g.info, cs, w >= 2 ? pend : nullptr,
                                std::make_integer_sequence<int, kW>{});
    if (w < 2) {  // no column 1 in this (last, narrow) panel: the flag goes now
      if (pend != nullptr) drain();
      __syncthreads();
      if (pend != nullptr && t == 0) set_flag(pend);
    }
    pend = nullptr;
    if (more && t == 0) {
      int ok = 1;
      if (pre == 0) {  // not published yet: bounded poll
        const unsigned long long t0 = rtc();
        while (__hip_atomic_load(&g.flags[np + j + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
          if (__hip_atomic_load(g.info + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
              rtc() - t0 > kSpinTicks) {
            __hip_atomic_store(g.info + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ok = 0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      sh.ok[j & 1] = ok;
    }
    __syncthreads();  // prow / sel complete; poll result visible
    stamp(g, j * 8 + 1);
    if (more && !sh.ok[j & 1]) return;

    // strip j+1 (steps < j applied by its updater): the TRSM right-hand sides
    // (the 16 pivot rows) and slot 0 are issued BEFORE any store, so waiting
    // for them never waits for the multiplier stores (in-order completion)
    double x = 0.0;
    u32x4 sv[4];  // first half (columns 0..7) of the next slot, in flight
    const __amdgpu_buffer_rsrc_t rh = rsrc(g.hbuf + (int64_t)(j + 1) * (kPanelBytes / 8), kPanelBytes);
    if (more) {
      if (t < 256) {
        const int J = t & 15, cc = t >> 4;
        const int pj = sh.sel[J];
        x = ld64(rh, tvo<R>(pj % NT) + soff(pj / NT, cc >> 1) + (cc & 1) * 8);
      }
#pragma unroll
      for (int cp = 0; cp < 4; ++cp) sv[cp] = ld128(rh, vo + soff(0, cp), 0);
    }
    // publish panel j: pivot rows (L11 | U11), pivots, U11 into work
    const __amdgpu_buffer_rsrc_t rp = rsrc(g.pbuf + (int64_t)j * 256, 256 * 8);
    if (t < 256) {
      const int J = t >> 4, c = t & 15;
      const double v = sh.prow[J][c];
      const int pj = sh.sel[J];
      st64(rp, t * 8, J < w ? v : 0.0);
      if (J < w && c >= J && c < w) g.work[(int64_t)pj * g.ldw + k0 + c] = v;
      if (J < w && c == 0) {
        st32(rpiv, (k0 + J) * 4, pj);
        st32(rps, (j * 32 + J) * 4, pj);
      }
    }
    const __amdgpu_buffer_rsrc_t rl = rsrc(g.lbuf + (int64_t)j * (kPanelBytes / 8), kPanelBytes);
    stamp(g, j * 8 + 2);
    if (!more) {
      // last panel (possibly narrow): phantom columns carry no multipliers
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int c = 0; c < kW; ++c) a[i][c] = c < w ? a[i][c] : 0.0;
#pragma unroll
      for (int i = 0; i < R; ++i)
#pragma unroll
        for (int cp = 0; cp < 8; ++cp) st128(rl, vo + soff(i, cp), 0, a[i][2 * cp], a[i][2 * cp + 1]);
      drain();
      __syncthreads();
      if (t == 0) set_flag(&g.flags[j]);
      break;
    }
    stamp(g, j * 8 + 3);

    // apply step j to strip j+1: U12 = L11^-1 x (DPP TRSM), then a rank-16
    // update of every slot with U12 from the scalar cache; the result is the
    // next panel, in the registers the factorisation uses
    const int k1 = k0 + kW;
    const int w1 = min(kW, n - k1);
    double* ut = g.ubuf + ((int64_t)j * (np + 1) + (j + 1)) * 256;
    if (t < 256) {
      const int J = t & 15, cc = t >> 4;
      double lrow[kW];
#pragma unroll
      for (int I = 0; I < kW; ++I) lrow[I] = sh.prow[J][I];
      trsm(x, lrow, J, std::make_integer_sequence<int, kW>{});
      ut[cc * kW + J] = x;
      if (cc < w1) g.work[(int64_t)sh.sel[J] * g.ldw + k1 + cc] = x;
    }
    drain();
    __syncthreads();
    stamp(g, j * 8 + 4);
    warm_u12(ut);
    // each slot's multipliers are published right after they are consumed,
    // so the stores drain under the update of the next slots
    // registers: the panel (R x 16) + one slot being updated + half a slot
    // in flight; the slot's second half is loaded at its start and lands
    // while its first 8 columns are updated
    sfor<R>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      double s[kW];
      u32x4 hi[4];
#pragma unroll
      for (int cp = 0; cp < 4; ++cp) hi[cp] = ld128(rh, vo + soff(i, 4 + cp), 0);
#pragma unroll
      for (int cp = 0; cp < 4; ++cp) {
        s[2 * cp] = mkd(sv[cp].x, sv[cp].y);
        s[2 * cp + 1] = mkd(sv[cp].z, sv[cp].w);
        s[8 + 2 * cp] = mkd(hi[cp].x, hi[cp].y);
        s[8 + 2 * cp + 1] = mkd(hi[cp].z, hi[cp].w);
      }
      if constexpr (i + 1 < R) {
#pragma unroll
        for (int cp = 0; cp < 4; ++cp) sv[cp] = ld128(rh, vo + soff(i + 1, cp), 0);
      }
      rank16(s, a[i], ut, kW);
#pragma unroll
      for (int cp = 0; cp < 8; ++cp) st128(rl, vo + soff(i, cp), 0, a[i][2 * cp], a[i][2 * cp + 1]);
#pragma unroll
      for (int c = 0; c < kW; ++c) a[i][c] = s[c];
    });
    stamp(g, j * 8 + 5);
    pend = &g.flags[j];  // drained and set behind column 1 of the next panel
    stamp(g, j * 8 + 6);
  }
}

// ---- updaters: one register-resident strip each --------------------------

template <int NT, int R>
__device__ __forceinline__ void updater(const Args& g, Shared& sh, int s) {
  const int t = threadIdx.x, lane = t & 63;
  const int vo = tvo<R>(t);
  const int n = g.n, np = g.np;
  constexpr int kPanelBytes = R * 8 * NT * 16;
  const bool bstrip = s == np;
  const int c0 = bstrip ? n : kW * s;
  const int ws = bstrip ? 1 : min(kW, n - c0);
  const int last = bstrip ? np - 1 : s - 2;  // step s-1 is applied by the engine
  double sr[R][kW];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const double* rp = g.src + (int64_t)min(t + i * NT, n - 1) * g.lds + c0;
#pragma unroll
    for (int c = 0; c < kW; ++c) sr[i][c] = rp[min(c, ws - 1)];
  }
  const __amdgpu_buffer_rsrc_t rpiv = rsrc(g.piv, (uint32_t)n * 4);
  const __amdgpu_buffer_rsrc_t rps = rsrc(g.pslot, (uint32_t)np * 128);
  for (int j = 0; j <= last; ++j) {
    if (!wait_flag(&g.flags[j], g.info + 1, sh, j & 1, 2)) return;
    stamp(g, 8 * np + 2 * (s * np + j));
    const int k0 = kW * j;
    const int wp = min(kW, n - k0);
    // lane J (mod 16) holds the pivot row of column k0 + J
    int pv = g.pslot_mode ? ld32(rps, (j * 32 + min(lane & 15, wp - 1)) * 4)
                          : ld32(rpiv, (k0 + min(lane & 15, wp - 1)) * 4);
    // a pivot row outside the system is a broken hand-off: report it (code
    // 8) and never store through it
    if (pv < 0 || pv >= n) {
      __hip_atomic_store(g.info + 1, 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pv = 0;
    }
    const __amdgpu_buffer_rsrc_t rp = rsrc(g.pbuf + (int64_t)j * 256, 256 * 8);
    if (t < 128) {
      const u32x4 v = ld128(rp, t * 16, 0);
      reinterpret_cast<double2*>(&sh.prow[0][0])[t] = make_double2(mkd(v.x, v.y), mkd(v.z, v.w));
    }
    // owners of this step's pivot rows hand their strip values to the TRSM
#pragma unroll
    for (int J = 0; J < kW; ++J) {
      const int pj = __builtin_amdgcn_readlane(pv, J);
      if (J < wp && t == pj % NT) {
#pragma unroll
        for (int i = 0; i < R; ++i)
          if (pj / NT == i) {
            put_row(reinterpret_cast<double2*>(&sh.xs[J][0]), sr[i]);
          }
      }
    }
    const __amdgpu_buffer_rsrc_t rl = rsrc(g.lbuf + (int64_t)j * (kPanelBytes / 8), kPanelBytes);
    u32x4 lv[8];
#pragma unroll
    for (int cp = 0; cp < 8; ++cp) lv[cp] = ld128(rl, vo + soff(0, cp), 0);
    __syncthreads();
    double* ut = g.ubuf + ((int64_t)j * (np + 1) + s) * 256;
    if (t < 256) {
      const int J = t & 15, cc = t >> 4;
      double lrow[kW];
#pragma unroll
      for (int I = 0; I < kW; ++I) lrow[I] = sh.prow[J][I];
      double x = J < wp ? sh.xs[J][cc] : 0.0;
      trsm(x, lrow, J, std::make_integer_sequence<int, kW>{});
      ut[cc * kW + J] = x;
      if (J < wp && cc < ws) g.work[(int64_t)pv * g.ldw + c0 + cc] = x;  // pv: pivot row of J
    }
    drain();
    __syncthreads();
    warm_u12(ut);
    sfor<R>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      double L[kW];
#pragma unroll
      for (int cp = 0; cp < 8; ++cp) {
        L[2 * cp] = mkd(lv[cp].x, lv[cp].y);
        L[2 * cp + 1] = mkd(lv[cp].z, lv[cp].w);
      }
      if constexpr (i + 1 < R) {
#pragma unroll
        for (int cp = 0; cp < 8; ++cp) lv[cp] = ld128(rl, vo + soff(i + 1, cp), 0);
      }
      rank16(sr[i], L, ut, ws);
    });
    stamp(g, 8 * np + 2 * (s * np + j) + 1);
  }
  if (!bstrip) {
    // hand the strip (steps 0..s-2 applied) to the engine
    const __amdgpu_buffer_rsrc_t rh = rsrc(g.hbuf + (int64_t)s * (kPanelBytes / 8), kPanelBytes);
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int cp = 0; cp < 8; ++cp) st128(rh, vo + soff(i, cp), 0, sr[i][2 * cp], sr[i][2 * cp + 1]);
    drain();
    __syncthreads();
    if (t == 0) set_flag(&g.flags[np + s]);
  }
}

// Up to 2 slots two workgroups may share a CU (128 VGPRs); 3 and 4 slots (the
// n <= 1536 / 2048 engines: np + 1 <= 129 workgroups, one per CU) get the
// whole 256-VGPR budget -- with (NT, 2) the 4-slot engine spilled 137 VGPRs
// to scratch (profiles/graph_recapture.txt: resident 2048 5.6 ms).
template <int NT, int R, int MODE>
__global__ __launch_bounds__(NT, NT == 512 && R <= 2 ? 2 : 1) void rlu_kernel(Args g) {
  __shared__ Shared sh;
  if (blockIdx.x == 0)
    engine<NT, R, MODE>(g, sh);
  else
    updater<NT, R>(g, sh, (int)blockIdx.x);
}

// Workspace of the resident LU for order n (bytes, 256-aligned pieces).
struct Layout {
  int NT = 0, R = 0, np = 0;
  size_t flags = 0, lbuf = 0, pbuf = 0, ubuf = 0, hbuf = 0, pslot = 0, total = 0;
};

Layout layout(int64_t n, int NT) {
  Layout L;
  if (n < 1 || n > 2048 || (NT != 512 && NT != 1024)) return Layout{};
  L.NT = NT;
  L.R = (int)((n + NT - 1) / NT);
  L.np = (int)((n + kW - 1) / kW);
  auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
  const size_t panel = (size_t)L.R * 8 * NT * 16;
  size_t off = 0;
  L.flags = off;
  off += up(sizeof(unsigned) * (2 * (size_t)L.np + 2));
  L.lbuf = off;
  off += up(panel * L.np);
  L.pbuf = off;
  off += up(sizeof(double) * 256 * (size_t)L.np);
  L.ubuf = off;
  off += up(sizeof(double) * 256 * (size_t)L.np * (L.np + 1));
  L.hbuf = off;
  off += up(panel * (L.np + 1));
  L.pslot = off;
  off += up((size_t)128 * L.np);
  L.total = off;
  return L;
}

}  // namespace
}  // namespace rlu

int64_t rlu_max_n() { return 2048; }

// The np + 1 workgroups of the resident LU hand panels and strips to each
// other through flags: they must all be resident at once.
// Workgroup size of the resident LU: 512 threads (1..4 register slots).
// (1024 threads -- 2 slots instead of 3-4 above 1024 rows -- spilled: 6.8 ms
// for the 2048 solve, profiles/headline_2048_r4.md.)
int rlu_threads(int64_t) { return 512; }

bool rlu_coresident(int64_t n) {
  using namespace rlu;
  const Layout L = layout(n, rlu_threads(n));
  if (!L.R) return false;
  int per = 0;
  hipError_t e = hipSuccess;
  if (L.R == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, rlu_kernel<512, 1, 1>, 512, 0);
  else if (L.R == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, rlu_kernel<512, 2, 1>, 512, 0);
  else if (L.R == 3) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, rlu_kernel<512, 3, 1>, 512, 0);
  else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, rlu_kernel<512, 4, 1>, 512, 0);
  return e == hipSuccess && coresident(per, L.np + 1);
}

size_t rlu_workspace_bytes(int64_t n) {
  // the larger of the two shapes, so a plan's workspace fits either
  return std::max(rlu::layout(n, 512).total, rlu::layout(n, 1024).total);
}

// Factor the augmented system src (n x (n+1), ld lds; NULL = work already
// holds it) into work (U rows at their physical positions, y in column n),
// with the pivot row of every column in piv.  ws: rlu_workspace_bytes(n)
// bytes of device memory.  info must be zeroed by the caller.
WordFill rlu_flags_fill(int64_t n, void* ws) {
  const rlu::Layout L = rlu::layout(n, rlu_threads(n));
  return WordFill{static_cast<char*>(ws) + L.flags, L.R ? (size_t)(L.lbuf - L.flags) : 0, 0u};
}

int rlu_factor(const double* src, int64_t lds, double* work, int64_t ldw, int64_t n, int mode,
               int* piv, int* info, void* ws, hipStream_t s, unsigned long long* stamps, bool flags_ready) {
  using namespace rlu;
  const Layout L = layout(n, rlu_threads(n));
  if (!L.R) return GELIM_FAIL(GELIM_E_ARG, "rlu: n out of range (1..2048)");
  char* base = static_cast<char*>(ws);
  Args a{};
  a.src = src ? src : work;
  a.lds = src ? lds : ldw;
  a.work = work;
  a.ldw = ldw;
  a.n = (int)n;
  a.np = L.np;
  a.piv = piv;
  a.info = info;
  a.flags = reinterpret_cast<unsigned*>(base + L.flags);
  a.lbuf = reinterpret_cast<double*>(base + L.lbuf);
  a.pbuf = reinterpret_cast<double*>(base + L.pbuf);
  a.ubuf = reinterpret_cast<double*>(base + L.ubuf);
  a.hbuf = reinterpret_cast<double*>(base + L.hbuf);
  a.pslot = reinterpret_cast<int*>(base + L.pslot);
  a.pslot_mode = 1;
  a.stamps = stamps;
  if (!flags_ready) GELIM_TRY(zero_async(a.flags, L.lbuf - L.flags, s));
  const dim3 grid((unsigned)(L.np + 1)), block((unsigned)L.NT);
  const bool part = mode == GELIM_PIVOT_PARTIAL;
  if (L.R == 1) {
    if (part) hipLaunchKernelGGL((rlu_kernel<512, 1, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((rlu_kernel<512, 1, 0>), grid, block, 0, s, a);
  } else if (L.R == 2) {
    if (part) hipLaunchKernelGGL((rlu_kernel<512, 2, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((rlu_kernel<512, 2, 0>), grid, block, 0, s, a);
  } else if (L.R == 3) {
    if (part) hipLaunchKernelGGL((rlu_kernel<512, 3, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((rlu_kernel<512, 3, 0>), grid, block, 0, s, a);
  } else {
    if (part) hipLaunchKernelGGL((rlu_kernel<512, 4, 1>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((rlu_kernel<512, 4, 0>), grid, block, 0, s, a);
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace gelim

// Diagnostic: factor a random n x (n+1) system twice (the second run with
// phase stamps) and return the raw stamps: engine [np][8] then updaters
// [np+1][np][2] (start, end of each applied step), 10 ns ticks.
extern "C" int gelim_debug_rlu_stamps(int64_t n, unsigned long long* out, int64_t out_len) {
  using namespace gelim;
  const int64_t np = (n + 15) / 16;
  const int64_t need = 8 * np + 2 * (np + 1) * np + 8;
  if (out_len < need) return GELIM_FAIL(GELIM_E_ARG, "debug_rlu_stamps: out too small");
  const int64_t ld = (n + 1 + 7) / 8 * 8;
  double *A = nullptr, *W = nullptr;
  int *piv = nullptr, *info = nullptr;
  void* ws = nullptr;
  unsigned long long* st = nullptr;
  HIP_TRY(hipMalloc((void**)&A, sizeof(double) * n * ld));
  HIP_TRY(hipMalloc((void**)&W, sizeof(double) * n * ld));
  HIP_TRY(hipMalloc((void**)&piv, sizeof(int) * (n + 64)));
  HIP_TRY(hipMalloc((void**)&info, 16));
  HIP_TRY(hipMalloc(&ws, rlu_workspace_bytes(n)));
  HIP_TRY(hipMalloc((void**)&st, sizeof(unsigned long long) * need));
  HIP_TRY(hipMemset(st, 0, sizeof(unsigned long long) * need));
  GELIM_TRY(gelim_gpu_init_random(A, ld, n, 1234, nullptr));
  GELIM_TRY(gelim_gpu_init_rhs(A, ld, n, nullptr));
  for (int rep = 0; rep < 2; ++rep) {
    HIP_TRY(hipMemset(info, 0, 16));
    GELIM_TRY(rlu_factor(A, ld, W, ld, n, GELIM_PIVOT_PARTIAL, piv, info, ws, nullptr, rep ? st : nullptr, false));
    HIP_TRY(hipDeviceSynchronize());
  }
  HIP_TRY(hipMemcpy(out, st, sizeof(unsigned long long) * need, hipMemcpyDeviceToHost));
  (void)hipFree(A);
  (void)hipFree(W);
  (void)hipFree(piv);
  (void)hipFree(info);
  (void)hipFree(ws);
  (void)hipFree(st);
  return GELIM_OK;
}
