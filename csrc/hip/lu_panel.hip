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
// How (MI355X-first): ONE workgroup of 1024 threads (16 wave64s) holds the
// whole panel in VGPRs — thread t owns rows t, t+1024, ... (R rows x W
// columns = 32 doubles = 64 VGPRs per lane) — so every column step is pure
// on-chip work with a SINGLE workgroup barrier:
//   1. each lane scans its rows, a DPP/shuffle wave arg-max picks the wave's
//      candidate, the winning lane writes its whole candidate row (W doubles)
//      into LDS and the owner of row j writes row j;
//   2. __syncthreads();
//   3. every wave re-reduces the 16 candidates itself (no second barrier),
//      reads the pivot row straight from the LDS slot of the winning wave,
//      exchanges rows j/p in registers and applies the rank-1 update.
// LDS slots are double-buffered by column parity, which is what makes the
// single barrier per column race-free.  The panel is read and written exactly
// once (coalesced 16-byte loads per row).
#include <hip/hip_runtime.h>

#include <utility>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / dev::kWave;

struct PanelLds {
  // slots double-buffered by column parity (one barrier per column)
  template <int W>
  struct T {
    double cand_row[2][kWaves][W];
    double rowj[2][W];
    double cand_val[2][kWaves];
    int cand_idx[2][kWaves];
    int piv[W];
  };
};

// Value barrier: stops LLVM from folding a select over register-array
// elements into a dynamically indexed load/store, which would demote the whole
// array to scratch memory.
__device__ __forceinline__ double opaque(double x) {
  asm volatile("" : "+v"(x));
  return x;
}

// One column step j = J of the panel (J is a compile-time constant so every
// register index below is static — a runtime j would spill a[][] to scratch).
template <int R, int W, int J>
__device__ __forceinline__ void panel_step(double (&a)[R][W], typename PanelLds::T<W>& sh, int t,
                                           int lane, int wave, int m, int w, int row0, int mode,
                                           int* __restrict__ info) {
  if (J >= w) return;  // uniform across the workgroup
  constexpr int par = J & 1;

  // 1. local + wave arg-max over rows >= J of column J
  double best = -1.0;
  int bidx = INT_MAX;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
    if (lr >= J && lr < m) {
      const double key = dev::pivot_key(a[i][J], lr == J, mode);
      if (key > best) {  // rows visited in increasing order: '>' keeps the lowest
        best = key;
        bidx = lr;
      }
    }
  }
  dev::wave_argmax(best, bidx);
  if (bidx != INT_MAX && (bidx & (kThreads - 1)) == t) {
    const int ip = bidx / kThreads;
    // branchless select keeps every register index static (no scratch)
#pragma unroll
    for (int c = 0; c < W; ++c) {
      double v = opaque(a[0][c]);
#pragma unroll
      for (int i = 1; i < R; ++i) v = (i == ip) ? opaque(a[i][c]) : v;
      sh.cand_row[par][wave][c] = v;
    }
  }
  if (lane == 0) {
    sh.cand_val[par][wave] = best;
    sh.cand_idx[par][wave] = bidx;
  }
  if (t == J) {  // row J lives in thread J, slot 0 (J < W <= 32)
#pragma unroll
    for (int c = 0; c < W; ++c) sh.rowj[par][c] = a[0][c];
  }
  __syncthreads();

  // 2. block winner, recomputed by every wave (no second barrier)
  double gv = (lane < kWaves) ? sh.cand_val[par][lane] : -1.0;
  int gi = (lane < kWaves) ? sh.cand_idx[par][lane] : INT_MAX;
  dev::group_argmax(gv, gi, kWaves);
  gv = __shfl(gv, 0, dev::kWave);
  const int p = __shfl(gi, 0, dev::kWave);
  const int pw = (p & (kThreads - 1)) >> 6;  // wave that published the pivot row
  const double* u = sh.cand_row[par][pw];  // pivot row, read from LDS (broadcast)
  const double d = u[J];
  if (t == 0) {
    sh.piv[J] = p;
    if (gv <= 0.0 && info && *info == 0) *info = row0 + J + 1;  // zero pivot
  }

  // 3. exchange rows J and p in registers (whole panel rows: L moves too)
  if (p != J) {
    if (t == J) {
#pragma unroll
      for (int c = 0; c < W; ++c) a[0][c] = sh.cand_row[par][pw][c];
    }
    if ((p & (kThreads - 1)) == t) {
      const int ip = p / kThreads;
#pragma unroll
      for (int c = 0; c < W; ++c) {
        const double v = sh.rowj[par][c];
#pragma unroll
        for (int i = 0; i < R; ++i) a[i][c] = opaque((i == ip) ? v : opaque(a[i][c]));
      }
    }
  }

  // 4. multipliers + rank-1 update of the rows below J
  const double rd = (d != 0.0) ? 1.0 / d : 0.0;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
    if (lr > J && lr < m) {
      const double l = a[i][J] * rd;
      a[i][J] = l;
#pragma unroll
      for (int c = J + 1; c < W; ++c) a[i][c] -= l * u[c];
    }
  }
}

template <int R, int W, int... J>
__device__ __forceinline__ void panel_steps(double (&a)[R][W], typename PanelLds::T<W>& sh, int t,
                                            int lane, int wave, int m, int w, int row0, int mode,
                                            int* info, std::integer_sequence<int, J...>) {
  (panel_step<R, W, J>(a, sh, t, lane, wave, m, w, row0, mode, info), ...);
}

template <int R, int W>
__global__ __launch_bounds__(kThreads) void panel_kernel(double* __restrict__ P, int64_t ldp,
                                                         int m, int w, int row0, int mode,
                                                         int* __restrict__ piv,
                                                         int* __restrict__ info) {
  __shared__ typename PanelLds::T<W> sh;
  const int t = threadIdx.x;
  const int lane = t & (dev::kWave - 1);
  const int wave = t >> 6;

  double a[R][W];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
    const double* src = P + (int64_t)lr * ldp;
#pragma unroll
    for (int c = 0; c < W; ++c) a[i][c] = (lr < m && c < w) ? src[c] : 0.0;
  }

  panel_steps<R, W>(a, sh, t, lane, wave, m, w, row0, mode, info,
                    std::make_integer_sequence<int, W>{});

#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int lr = t + i * kThreads;
    if (lr < m) {
      double* dst = P + (int64_t)lr * ldp;
#pragma unroll
      for (int c = 0; c < W; ++c)
        if (c < w) dst[c] = a[i][c];
    }
  }
  __syncthreads();
  if (t < w) piv[t] = sh.piv[t];
}

template <int R, int W>
int launch_panel(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode,
                 int* piv, int* info, hipStream_t s) {
  hipLaunchKernelGGL((panel_kernel<R, W>), dim3(1), dim3(kThreads), 0, s, P, ldp, (int)m,
                     (int)w, (int)row0, mode, piv, info);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// Widest register panel that fits 32 doubles per lane for m rows.
int64_t panel_width_for(int64_t m) {
  if (m <= 1024) return 32;
  if (m <= 2048) return 16;
  if (m <= 4096) return 8;
  if (m <= 8192) return 4;
  if (m <= 16384) return 2;
  return 0;
}

int panel_factor(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode,
                 int* piv, int* info, hipStream_t s) {
  if (m <= 0 || w <= 0 || w > m) return GELIM_FAIL(GELIM_E_ARG, "panel: bad m/w");
  if (m <= 1024 && w <= 32) return launch_panel<1, 32>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 2048 && w <= 16) return launch_panel<2, 16>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 4096 && w <= 8) return launch_panel<4, 8>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 8192 && w <= 4) return launch_panel<8, 4>(P, ldp, m, w, row0, mode, piv, info, s);
  if (m <= 16384 && w <= 2) return launch_panel<16, 2>(P, ldp, m, w, row0, mode, piv, info, s);
  return GELIM_FAIL(GELIM_E_ARG, "panel: m=" + std::to_string(m) + " w=" + std::to_string(w) +
                                     " exceeds the register-resident panel");
}

}  // namespace gelim

extern "C" int gelim_gpu_panel_factor(double* dP, int64_t ldp, int64_t m, int64_t w,
                                      int64_t row0, int pivot, int32_t* dpiv, int32_t* dinfo,
                                      void* stream) {
  return gelim::panel_factor(dP, ldp, m, w, row0, pivot, dpiv, dinfo, (hipStream_t)stream);
}

extern "C" int64_t gelim_gpu_panel_max_rows(int64_t w) {
  if (w <= 2) return 16384;
  if (w <= 4) return 8192;
  if (w <= 8) return 4096;
  if (w <= 16) return 2048;
  if (w <= 32) return 1024;
  return 0;
}
