// Panel factorisation for the blocked LU (the latency-critical part of
// Gaussian elimination on MI355X).
//
// What it computes: the reference's pivot search + row swap + elimination
// (getPivot / computeGauss, OpenMP_and_MPI/gauss_openmp/gauss_external_input.c
// :123-182) restricted to a tall m x w column panel, LAPACK-getf2 style:
// for j in 0..w-1: choose pivot row p >= j (PARTIAL: argmax |a|, ties to the
// lowest row; ZERO: reference internal rule), swap rows j and p across the
// panel, L[r][j] = a[r][j] / a[j][j], rank-1 update of the panel's remaining
// columns.
//
// How (MI355X-first): ONE workgroup of 256 threads — 4 wave64s, one per SIMD,
// so each wave owns the SIMD's whole 512-entry VGPR file — holds the panel in
// registers: thread t owns rows t, t+256, ... (R rows x W columns = up to 128
// doubles = 256 VGPRs per lane, 256 KiB per CU), so every column step is
// on-chip work with a SINGLE workgroup barrier:
//   1. each lane scans its rows; a DPP max-scan of the (order-preserving
//      integer) key followed by a DPP min-scan of the rows holding it gives
//      the wave's candidate (ties -> lowest row, like the reference's strict
//      '>'); the winning lane writes its whole candidate row into LDS and the
//      owner of row j writes row j;
//   2. __syncthreads();
//   3. every wave reduces the 4 wave candidates itself (no second barrier),
//      reads the pivot row from the LDS slot of the winning wave, exchanges
//      rows j/p in registers and applies the rank-1 update with fp64 FMAs.
// Fewer, fatter waves matter: with 16 waves the per-column overhead (reductions,
// LDS traffic, branches) was issued 4x per SIMD and dominated (4-5 us/column).
// LDS slots are double-buffered by column parity, which is what makes the
// single barrier per column race-free.  The panel is read and written exactly
// once (coalesced 16-byte loads per row).
#include <hip/hip_runtime.h>

#include <utility>
#include <vector>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kThreads = 256;  // 4 wave64s: one per SIMD, each with the full VGPR file
constexpr int kWaves = kThreads / dev::kWave;

template <int W>
struct alignas(16) PanelLds {
  // slots double-buffered by column parity (one barrier per column)
  double cand_row[2][kWaves][W];
  unsigned cand_key[2][kWaves][2];  // {hi, lo} of the wave's winning key
  unsigned cand_row_idx[2][kWaves];
  int sel[W];           // physical (original) row chosen at each step
  int pos_of[2 * W];    // compact row id -> compact position
  int row_at[2 * W];    // compact position -> compact row id
  int piv[W];
};

// Value barrier: stops LLVM from folding a select over register-array
// elements into a dynamically indexed access, which would demote the whole
// array to scratch memory.
__device__ __forceinline__ double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

// One column step j = J of the panel (J is a compile-time constant so every
// register index below is static — a runtime j would spill a[][] to scratch).
// Rows are never moved during the column loop ("logical pivoting"): a chosen
// row is retired via the per-lane `chosen` bit mask and keeps its place; the
// LAPACK interchange sequence is reconstructed once at the end.
template <int R, int W, int J>
__device__ __forceinline__ void panel_step(double (&a)[R][W], uint64_t& chosen, PanelLds<W>& sh,
                                           int t, int lane, int wave, int m, int w, int row0,
                                           int mode, int* __restrict__ info) {
  if (J >= w) return;  // uniform across the workgroup
  constexpr int par = J & 1;

  // 1. local candidate over this lane's live rows (not yet chosen, < m)
  uint64_t best = 0;
  unsigned brow = 0xffffffffu;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
    const bool ok = !((chosen >> i) & 1) && lr < m;
    // the reference's diagonal preference (ZERO rule) refers to the row that
    // currently sits at position J: physically row J unless it was chosen
    // earlier, in which case no row is "the diagonal" for that rule (a
    // deliberate, documented difference from a physical-swap run)
    const uint64_t key = ok ? dev::pivot_ukey(a[i][J], lr == J, mode) : 0;
    const bool better = key > best;  // increasing rows: '>' keeps the lowest row on ties
    best = better ? key : best;
    brow = better ? (unsigned)lr : brow;
  }
  // 2. wave arg-max: DPP max of the key, then DPP min of the rows holding it
  const uint64_t wkey = dev::wave_max_u64(best);
  // exact ties are rare: one ballot finds the single holder; only a real tie
  // pays the second (row-min) DPP chain (uniform branch)
  const uint64_t holders = __ballot(best == wkey);
  unsigned wrow;
  if (__popcll(holders) == 1)
    wrow = (unsigned)__builtin_amdgcn_readlane((int)brow, __ffsll((long long)holders) - 1);
  else
    wrow = dev::wave_min_u32(best == wkey ? brow : 0xffffffffu);
  if (wkey != 0 && (int)(wrow & (kThreads - 1)) == t) {
    const int ip = (int)(wrow / kThreads);
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
  __syncthreads();

  // 3. block winner from the 4 wave candidates (broadcast LDS reads)
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
  const int pw = (int)((p & (kThreads - 1)) >> 6);  // wave that published the pivot row
  const double* u = sh.cand_row[par][pw];
  const double d = u[J];
  if (t == 0) {
    sh.sel[J] = (int)p;
    if (gkey <= 1 && info && *info == 0) *info = row0 + J + 1;  // zero pivot
  }
  if ((int)(p & (kThreads - 1)) == t) chosen |= 1ull << (p / kThreads);

  // 4. multipliers + rank-1 update of every live row (retired rows get l = 0)
  const double rd = (d != 0.0) ? 1.0 / d : 0.0;
  double uc[W];
#pragma unroll
  for (int c = J + 1; c < W; ++c) uc[c] = u[c];
  double l[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const bool live = !((chosen >> i) & 1);
    l[i] = live ? a[i][J] * rd : 0.0;
    a[i][J] = live ? l[i] : a[i][J];
  }
  // column J+1 first: the next step's pivot search depends only on it
  if constexpr (J + 1 < W) {
#pragma unroll
    for (int i = 0; i < R; ++i) a[i][J + 1] = fma(-l[i], uc[J + 1], a[i][J + 1]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int c = J + 2; c < W; ++c) a[i][c] = fma(-l[i], uc[c], a[i][c]);
}

template <int R, int W, int... J>
__device__ __forceinline__ void panel_steps(double (&a)[R][W], uint64_t& chosen, PanelLds<W>& sh,
                                            int t, int lane, int wave, int m, int w, int row0,
                                            int mode, int* info, std::integer_sequence<int, J...>) {
  (panel_step<R, W, J>(a, chosen, sh, t, lane, wave, m, w, row0, mode, info), ...);
}

// LDS staging tile for the coalesced panel load/store: 256 rows x W doubles,
// 16-byte chunks XOR-swizzled by row so that the per-row ds_read_b128 /
// ds_write_b128 of 16 consecutive lanes hit distinct banks.
template <int W>
__device__ __forceinline__ int swz_chunk(int row, int ch) {
  constexpr int CH = W / 2;
  return ch ^ (row & (CH - 1));
}

extern __shared__ __attribute__((aligned(16))) char g_panel_dyn_lds[];

template <int R, int W>
__device__ __forceinline__ void stage_in(double (&a)[R][W], const double* __restrict__ P,
                                         int64_t ldp, int m, int t) {
  constexpr int CH = W / 2;                    // chunks per row
  constexpr int ROWS_PER_PASS = kThreads / CH;  // rows per coalesced pass
  double2* tile = reinterpret_cast<double2*>(g_panel_dyn_lds);  // [kThreads][CH]
#pragma unroll
  for (int i = 0; i < R; ++i) {
    // coalesced: lane group of CH lanes reads one row's W doubles
    const int ch = t % CH;
#pragma unroll
    for (int pass = 0; pass < kThreads / ROWS_PER_PASS; ++pass) {
      const int rl = pass * ROWS_PER_PASS + t / CH;  // row within this slot
      const int lr = i * kThreads + rl;
      double2 v = make_double2(0.0, 0.0);
      if (lr < m) v = *reinterpret_cast<const double2*>(P + (int64_t)lr * ldp + 2 * ch);
      tile[rl * CH + swz_chunk<W>(rl, ch)] = v;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const double2 v = tile[t * CH + swz_chunk<W>(t, c)];
      a[i][2 * c] = v.x;
      a[i][2 * c + 1] = v.y;
    }
    __syncthreads();
  }
}

template <int R, int W>
__device__ __forceinline__ void stage_out(const double (&a)[R][W], const int (&dest)[R],
                                          double* __restrict__ P, int64_t ldp, int m, int t) {
  constexpr int CH = W / 2;
  constexpr int ROWS_PER_PASS = kThreads / CH;
  double2* tile = reinterpret_cast<double2*>(g_panel_dyn_lds);
  int* dst_row = reinterpret_cast<int*>(g_panel_dyn_lds + sizeof(double2) * kThreads * CH);
#pragma unroll
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) tile[t * CH + swz_chunk<W>(t, c)] = make_double2(a[i][2 * c], a[i][2 * c + 1]);
    dst_row[t] = dest[i];
    __syncthreads();
    const int ch = t % CH;
#pragma unroll
    for (int pass = 0; pass < kThreads / ROWS_PER_PASS; ++pass) {
      const int rl = pass * ROWS_PER_PASS + t / CH;
      const int lr = i * kThreads + rl;
      if (lr < m)
        *reinterpret_cast<double2*>(P + (int64_t)dst_row[rl] * ldp + 2 * ch) =
            tile[rl * CH + swz_chunk<W>(rl, ch)];
    }
    __syncthreads();
  }
}

// Diagnostic stamps (separate build of the same kernel, never used by the
// solver): thread 0 records s_memtime at phase boundaries into `stamps`.
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int R, int W, bool STAMP = false>
__global__ __launch_bounds__(kThreads) void panel_kernel(double* __restrict__ P, int64_t ldp,
                                                         int m, int w, int row0, int mode,
                                                         int* __restrict__ piv,
                                                         int* __restrict__ info,
                                                         unsigned long long* __restrict__ stamps = nullptr) {
  static_assert(R <= 64, "chosen mask is 64 bits");
  __shared__ PanelLds<W> sh;
  const int t = threadIdx.x;
  const int lane = t & (dev::kWave - 1);
  const int wave = t >> 6;

  unsigned long long t0 = 0;
  if constexpr (STAMP) t0 = stamp_now();
  double a[R][W];
  // full-width panels with 16-byte aligned rows are staged through LDS so
  // that global loads are coalesced (8 lanes per 128-byte row segment)
  const bool staged = (w == W) && (W % 2 == 0) && ((((uintptr_t)P) & 15) == 0) && (ldp % 2 == 0);
  if (staged) {
    stage_in<R, W>(a, P, ldp, m, t);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * kThreads;
      const double* src = P + (int64_t)min(lr, m - 1) * ldp;  // clamped: no divergent loads
#pragma unroll
      for (int c = 0; c < W; ++c) {
        const double v = src[min(c, w - 1)];
        a[i][c] = (lr < m && c < w) ? v : 0.0;
      }
    }
  }
  uint64_t chosen = 0;
  if constexpr (STAMP) {
    __syncthreads();
    if (t == 0) {
      stamps[0] = t0;
      stamps[1] = stamp_now();
    }
  }

  panel_steps<R, W>(a, chosen, sh, t, lane, wave, m, w, row0, mode, info,
                    std::make_integer_sequence<int, W>{});
  if constexpr (STAMP) {
    if (t == 0) stamps[2] = stamp_now();
  }

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
  }
  __syncthreads();

  // write back every physical row to its final position
  int dest[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
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
    stage_out<R, W>(a, dest, P, ldp, m, t);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int lr = t + i * kThreads;
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
      stamps[3] = stamp_now();
      stamps[4] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

template <int W>
constexpr size_t stage_bytes() {
  return sizeof(double) * kThreads * W + sizeof(int) * kThreads;
}

template <int R, int W>
int launch_panel(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode,
                 int* piv, int* info, hipStream_t s) {
  hipLaunchKernelGGL((panel_kernel<R, W>), dim3(1), dim3(kThreads), stage_bytes<W>(), s, P, ldp,
                     (int)m, (int)w, (int)row0, mode, piv, info, nullptr);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// Widest register panel for m rows: R x W = 128 doubles (256 VGPRs) per lane,
// 256 lanes -> 256 KiB of panel held on one CU.
int64_t panel_width_for(int64_t m) {
  if (m <= 2048) return 16;
  if (m <= 4096) return 8;
  if (m <= 8192) return 4;
  if (m <= 16384) return 2;
  return 0;
}

int panel_factor(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode,
                 int* piv, int* info, hipStream_t s) {
  if (m <= 0 || w <= 0 || w > m) return GELIM_FAIL(GELIM_E_ARG, "panel: bad m/w");
  if (m <= 256 && w <= 16) return launch_panel<1, 16>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 512 && w <= 16) return launch_panel<2, 16>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 1024 && w <= 16) return launch_panel<4, 16>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 2048 && w <= 16) return launch_panel<8, 16>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 4096 && w <= 8) return launch_panel<16, 8>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 8192 && w <= 4) return launch_panel<32, 4>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 16384 && w <= 2) return launch_panel<64, 2>(P, ldp, m, w, row0, mode, piv, info, s);
  return GELIM_FAIL(GELIM_E_ARG, "panel: m=" + std::to_string(m) + " w=" + std::to_string(w) +
                                     " exceeds the register-resident panel");
}

}  // namespace gelim

extern "C" int gelim_gpu_panel_factor(double* dP, int64_t ldp, int64_t m, int64_t w,
                                      int64_t row0, int pivot, int32_t* dpiv, int32_t* dinfo,
                                      void* stream) {
  return gelim::panel_factor(dP, ldp, m, w, row0, pivot, dpiv, dinfo, (hipStream_t)stream);
}

// Diagnostic: run the stamped panel kernel once on a random m x 16 panel and
// return {t_load, t_steps, t_store} in shader cycles (plus total).
extern "C" int gelim_debug_panel_stamps(int64_t m, int64_t w, unsigned long long* out4) {
  using namespace gelim;
  double* P = nullptr;
  int *piv = nullptr, *info = nullptr;
  unsigned long long* st = nullptr;
  HIP_TRY(hipMalloc((void**)&P, sizeof(double) * m * 16));
  HIP_TRY(hipMalloc((void**)&piv, sizeof(int) * 64));
  HIP_TRY(hipMalloc((void**)&info, 16));
  HIP_TRY(hipMalloc((void**)&st, 64));
  std::vector<double> h(m * 16);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 997.0 - 0.5;
  HIP_TRY(hipMemcpy(P, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(info, 0, 16));
  for (int rep = 0; rep < 3; ++rep) {
    if (m <= 256) hipLaunchKernelGGL((panel_kernel<1, 16, true>), 1, kThreads, stage_bytes<16>(), 0, P, 16, (int)m, (int)w, 0, 1, piv, info, st);
    else if (m <= 1024) hipLaunchKernelGGL((panel_kernel<4, 16, true>), 1, kThreads, stage_bytes<16>(), 0, P, 16, (int)m, (int)w, 0, 1, piv, info, st);
    else hipLaunchKernelGGL((panel_kernel<8, 16, true>), 1, kThreads, stage_bytes<16>(), 0, P, 16, (int)m, (int)w, 0, 1, piv, info, st);
    HIP_TRY(hipDeviceSynchronize());
  }
  unsigned long long hs[8];
  HIP_TRY(hipMemcpy(hs, st, 64, hipMemcpyDeviceToHost));
  out4[0] = hs[1] - hs[0];
  out4[1] = hs[2] - hs[1];
  out4[2] = hs[3] - hs[2];
  out4[3] = hs[3] - hs[0];
  (void)hipFree(P); (void)hipFree(piv); (void)hipFree(info); (void)hipFree(st);
  return GELIM_OK;
}

extern "C" int64_t gelim_gpu_panel_max_rows(int64_t w) {  // rows per width
  if (w <= 2) return 16384;
  if (w <= 4) return 8192;
  if (w <= 8) return 4096;
  if (w <= 16) return 2048;
  return 0;
}
