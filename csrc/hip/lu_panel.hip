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

#include <utility>
#include <vector>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kMaxWaves = 8;

template <int W>
struct alignas(16) PanelLds {
  double cand_row[2][kMaxWaves][W];    // each wave's winning row (parity-buffered)
  unsigned cand_key[2][kMaxWaves][2];  // {hi, lo} of the wave's winning key
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

template <int NT, int R, int W, int MODE, bool STAMP>
struct Panel {
  static constexpr int kWaves = NT / dev::kWave;
  static_assert(kWaves <= kMaxWaves, "too many waves");
  static_assert(R <= 64, "chosen mask is 64 bits");

  template <int J>
  static __device__ __forceinline__ void stamp(StepStamps& ss, int slot) {
    if constexpr (STAMP) {
      if (J == 4) ss.v[slot] = stamp_now();
    }
  }

  // One column step J (compile time, so every register index is static).
  template <int J>
  static __device__ __forceinline__ void step(double (&a)[R][W], uint64_t& chosen,
                                              PanelLds<W>& sh, int t, int lane, int wave, int m,
                                              int w, int row0, int* __restrict__ info,
                                              StepStamps& ss) {
    if (J >= w) return;  // uniform across the workgroup
    constexpr int par = J & 1;
    stamp<J>(ss, 0);

    // 1. local candidate over this lane's live rows (not yet chosen, < m)
    uint64_t best = 0;
    unsigned brow = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      const bool ok = !((chosen >> i) & 1) && lr < m;
      // ZERO rule: the "diagonal" is physical row J (a row chosen earlier is
      // never the diagonal here — documented difference from a physical-swap
      // run; PARTIAL pivoting, the accuracy-relevant rule, is exact)
      const uint64_t key = dev::pivot_ukey_t<MODE>(a[i][J], lr == J, ok);
      const bool better = key > best;  // increasing rows: '>' keeps the lowest row on ties
      best = better ? key : best;
      brow = better ? (unsigned)lr : brow;
    }

    // 2. wave arg-max: DPP max of the high word, one ballot; exact fallback
    const unsigned bhi = (unsigned)(best >> 32);
    const unsigned hmax = dev::wave_max_u32(bhi);
    const uint64_t holders = __ballot(bhi == hmax);
    uint64_t wkey;
    unsigned wrow;
    if (__popcll(holders) == 1) {
      const int wl = __ffsll((long long)holders) - 1;
      wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, wl);
      wkey = ((uint64_t)hmax << 32) | (unsigned)__builtin_amdgcn_readlane((int)(unsigned)best, wl);
    } else {
      wkey = dev::wave_max_u64(best);
      const uint64_t h2 = __ballot(best == wkey);
      if (__popcll(h2) == 1)
        wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, __ffsll((long long)h2) - 1);
      else
        wrow = dev::wave_min_u32(best == wkey ? brow : 0xffffffffu);
    }
    stamp<J>(ss, 1);

    // the lane holding the wave's winner publishes its row (uniform slot)
    if (wkey != 0 && (int)(wrow % NT) == t) {
      const int ip = (int)(wrow / NT);
#pragma unroll
      for (int i = 0; i < R; ++i)
        if (i == ip) {
#pragma unroll
          for (int c = 0; c < W; ++c) sh.cand_row[par][wave][c] = opaque(a[i][c]);
        }
    }
    if (lane == 0) {
      sh.cand_key[par][wave][0] = (unsigned)(wkey >> 32);
      sh.cand_key[par][wave][1] = (unsigned)wkey;
      sh.cand_row_idx[par][wave] = wrow;
    }
    stamp<J>(ss, 2);
    __syncthreads();
    stamp<J>(ss, 3);

    // 3. block winner from the per-wave candidates (broadcast LDS reads)
    uint64_t gkey = 0;
    unsigned p = 0xffffffffu;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) {
      const uint64_t k = ((uint64_t)sh.cand_key[par][q][0] << 32) | sh.cand_key[par][q][1];
      const unsigned r = sh.cand_row_idx[par][q];
      const bool better = k > gkey || (k == gkey && r < p);
      gkey = better ? k : gkey;
      p = better ? r : p;
    }
    const int pw = (int)((p % NT) >> 6);  // wave that published the pivot row
    const double* u = sh.cand_row[par][pw];
    const double d = u[J];
    const double rd = (d != 0.0) ? 1.0 / d : 0.0;
    double uc[W];
#pragma unroll
    for (int c = J + 1; c < W; ++c) uc[c] = u[c];
    if (t == 0) {
      sh.sel[J] = (int)p;
      if (gkey <= 1 && info && *info == 0) *info = row0 + J + 1;  // zero pivot
    }
    if ((int)(p % NT) == t) chosen |= 1ull << (p / NT);
    stamp<J>(ss, 4);

    // 4. multipliers + rank-1 update of every live row (retired rows: l = 0);
    //    column J+1 first — the next step's pivot search depends only on it
    double l[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const bool live = !((chosen >> i) & 1);
      l[i] = live ? a[i][J] * rd : 0.0;
      a[i][J] = live ? l[i] : a[i][J];
    }
    if constexpr (J + 1 < W) {
#pragma unroll
      for (int i = 0; i < R; ++i) a[i][J + 1] = fma(-l[i], uc[J + 1], a[i][J + 1]);
    }
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int c = J + 2; c < W; ++c) a[i][c] = fma(-l[i], uc[c], a[i][c]);
    if constexpr (STAMP) {
      if (J == 4) {
        asm volatile("" ::"v"(a[R - 1][W - 1]));
        ss.v[5] = stamp_now();
      }
    }
  }

  template <int... J>
  static __device__ __forceinline__ void steps(double (&a)[R][W], uint64_t& chosen,
                                               PanelLds<W>& sh, int t, int lane, int wave, int m,
                                               int w, int row0, int* info, StepStamps& ss,
                                               std::integer_sequence<int, J...>) {
    (step<J>(a, chosen, sh, t, lane, wave, m, w, row0, info, ss), ...);
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
};

template <int NT, int R, int W, int MODE, bool STAMP = false>
__global__ __launch_bounds__(NT) void panel_kernel(double* __restrict__ P, int64_t ldp, int m,
                                                   int w, int row0, int* __restrict__ piv,
                                                   int* __restrict__ info,
                                                   unsigned long long* __restrict__ stamps,
                                                   int* __restrict__ pairs) {
  using K = Panel<NT, R, W, MODE, STAMP>;
  __shared__ PanelLds<W> sh;
  const int t = threadIdx.x;
  const int lane = t & (dev::kWave - 1);
  const int wave = t >> 6;
  unsigned long long t0 = 0;
  if constexpr (STAMP) t0 = stamp_now();

  double a[R][W];
  // full-width panels with 16-byte aligned rows are staged through LDS so the
  // global loads are coalesced (W/2 lanes per row segment)
  const bool staged = (w == W) && (W % 2 == 0) && ((((uintptr_t)P) & 15) == 0) && (ldp % 2 == 0);
  if (staged) {
    K::stage_in(a, P, ldp, m, t);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * NT;
      const double* src = P + (int64_t)min(lr, m - 1) * ldp;  // clamped: no divergent loads
#pragma unroll
      for (int c = 0; c < W; ++c) {
        const double v = src[min(c, w - 1)];
        a[i][c] = (lr < m && c < w) ? v : 0.0;
      }
    }
  }
  uint64_t chosen = 0;
  unsigned long long t1 = 0;
  if constexpr (STAMP) {
    __syncthreads();
    t1 = stamp_now();
  }

  StepStamps ss{};
  K::steps(a, chosen, sh, t, lane, wave, m, w, row0, info, ss, std::make_integer_sequence<int, W>{});
  unsigned long long t2 = 0;
  if constexpr (STAMP) t2 = stamp_now();

  // Reconstruct LAPACK's sequential interchanges from the selection order.
  // Compact ids: rows < w keep their index; a chosen row >= w selected at
  // step j gets id w + j.  Compact positions use the same numbering (the
  // only positions >= w ever touched are original places of chosen rows).
  if (t == 0) {
    for (int x = 0; x < 2 * w; ++x) {
      sh.pos_of[x] = x;
      sh.row_at[x] = x;
    }
    for (int j = 0; j < w; ++j) {
      const int p = sh.sel[j];
      const int idp = p < w ? p : w + j;
      const int cur = sh.pos_of[idp];
      const int other = sh.row_at[j];
      sh.row_at[j] = idp;
      sh.row_at[cur] = other;
      sh.pos_of[idp] = j;
      sh.pos_of[other] = cur;
      sh.piv[j] = cur < w ? cur : sh.sel[cur - w];
    }
    // net row movement as (dst, src) pairs for the trailing-column kernels:
    // new_row[dst] = old_row[src] over the <= 2w touched rows
    if (pairs) {
      int np = 0;
      for (int x = 0; x < 2 * w; ++x) {
        // compact position w+j stands for actual position sel[j] only when
        // that row lies below the panel top (otherwise it is unused)
        if (x >= w && sh.sel[x - w] < w) continue;
        const int ap = x < w ? x : sh.sel[x - w];
        const int id = sh.row_at[x];
        const int ar = id < w ? id : sh.sel[id - w];
        if (ap != ar) {
          pairs[1 + 2 * np] = ap;
          pairs[2 + 2 * np] = ar;
          ++np;
        }
      }
      pairs[0] = np;
    }
  }
  __syncthreads();

  // final position of every physical row
  int dest[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * NT;
    int d = lr;
    int id = -1;
    if (lr < w) {
      id = lr;
    } else if (lr < m && ((chosen >> i) & 1)) {
      for (int j = 0; j < w; ++j)
        if (sh.sel[j] == lr) id = w + j;
    }
    if (id >= 0) {
      const int cp = sh.pos_of[id];
      d = cp < w ? cp : sh.sel[cp - w];
    }
    dest[i] = d;
  }
  if (staged) {
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
      for (int k = 0; k < 6; ++k) stamps[8 + k] = ss.v[k];
    }
  }
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
