// Back substitution U x = y on the GPU (the reference's solveGauss,
// Pthreads/Version-1/gauss_internal_input.c:212-227, a serial O(n^2) loop
// there).
//
// Default: ONE persistent launch (backsub_persist_kernel), row block b (64
// equations) in workgroup b, x produced bottom-up.  Round 5 form: every
// workgroup first forms W = T^-1 U[b, b+1] and W2 = T^-1 U[b, b+2] (T its
// diagonal triangle; all workgroups at once, off the chain); its compute
// waves accumulate U[b, c] x_c for c > b + 2 as the x_c land; a poller wave
// solves T v' = y_b - sum two chain steps ahead, and the chain itself is
// two 64 x 64 mat-vecs, x_b = v' - W2 x_{b+2} - W x_{b+1}.  x itself is the
// hand-off: pre-filled with a signalling-NaN sentinel, each value stored sc1
// and polled sc1 (no flag).  2048: 155 -> ~75 us per solve (4.8 -> ~1.8 us
// per block), profiles/backsub_r5.txt.
// Spins are bounded (200 ms) and report through an error word.
//
// Rows may be indirect: perm[i] is the row of U (and of y) that holds
// equation i -- the resident LU (rlu.hip) leaves U rows at their physical
// positions.  Without perm, row i is equation i.
//
// Fallback when the blocks cannot all be resident (more than 256 blocks,
// n > 16384): one launch per block (backsub_step_kernel).
#include <hip/hip_runtime.h>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr int kBS = 64;
constexpr int kMaxPersistBlocks = 256;
constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz

// Row of equation i; a row map entry outside [0, n) (a corrupt map, e.g. one
// left stale by an aborted factorisation) is clamped, never dereferenced --
// the persistent kernel reports it through its error word (code 7).
__device__ __forceinline__ int rowof(const int* perm, int i, int n) {
  return perm ? min(max(perm[i], 0), n - 1) : i;
}

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

template <typename T>
__global__ void copy_y_kernel(const T* __restrict__ U, int64_t ldu, const T* __restrict__ y,
                              int64_t incy, const int* __restrict__ perm, double* __restrict__ yw,
                              double* __restrict__ bnorm, int n, int unit) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int r = rowof(perm, i, n);
  const double v = (double)y[(int64_t)r * incy];
  yw[i] = v;
  if (bnorm) bnorm[i] = unit ? v : v / (double)U[(int64_t)r * ldu + i];
}

// Wave 0's copy of a diagonal block: lane l keeps equation i0+l's row
// (columns i0..i0+nb) and the reciprocal of its diagonal.
template <typename T>
__device__ __forceinline__ void load_diag(const T* __restrict__ U, int64_t ldu, const int* perm, int n, int i0,
                                          int nb, int unit, double (&row)[kBS], double& rinv) {
  const int l = threadIdx.x & 63;
  const int lc = min(l, nb - 1);
  const T* src = U + (int64_t)rowof(perm, i0 + lc, n) * ldu + i0;
#pragma unroll
  for (int c = 0; c < kBS; ++c) row[c] = dev::load_sel(src + min(c, nb - 1), l < nb && c < nb);
  rinv = unit ? 1.0 : 1.0 / (double)src[lc];
}

// One wave solves the nb x nb triangle: x_i broadcast with v_readlane (i is
// wave-uniform), so the serial chain is mul -> readlane -> fma per step.
__device__ __forceinline__ double solve_diag(const double (&row)[kBS], double rinv, double yv, int nb) {
  const int l = threadIdx.x & 63;
  double xv = 0.0;
#pragma unroll
  for (int i = kBS - 1; i >= 0; --i) {
    if (i < nb) {
      const double xi_l = yv * rinv;  // meaningful in lane i only
      const uint64_t b = __builtin_bit_cast(uint64_t, xi_l);
      const double xi = __builtin_bit_cast(
          double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), i) << 32) |
                      (unsigned)__builtin_amdgcn_readlane((int)b, i));
      if (l == i) xv = xi;
      yv = (l < i) ? fma(-row[i], xi, yv) : yv;
    }
  }
  return xv;
}

// ---- persistent form ---------------------------------------------------------
// x is pre-filled with a signalling-NaN sentinel (arithmetic only ever makes
// quiet NaNs), and every x value is its own hand-off: stored sc1 by its
// producer, polled with sc1 loads by its consumers (a data-tagged granule, no
// separate flag: one hop instead of payload -> drain -> flag -> poll).
constexpr uint64_t kXSent = 0x7ff4dead7ff4deadull;

__global__ void fill_sent_kernel(uint64_t* __restrict__ x, int n, int* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = kXSent;
  if (i == 0 && err) *err = 0;
}

// Wave-wide bounded poll until lanes < cw of x[c0 ..] are published; returns
// this lane's value.  false (and the error word set) when the spin ran out or
// another workgroup already gave up.
__device__ __forceinline__ bool poll_x(const double* __restrict__ x, int c0, int cw, int* err, bool nap,
                                       double& xl) {
  const int lane = __lane_id();
  const unsigned long long* p = reinterpret_cast<const unsigned long long*>(x + c0 + min(lane, cw - 1));
  uint64_t v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (__ballot(v == kXSent) != 0) {
    const unsigned long long t0 = rtc();
    for (int it = 0;; ++it) {
      if (nap) __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__ballot(v == kXSent) == 0) break;
      // every 16th probe: another workgroup gave up, or this spin ran out
      // (not every probe: the extra load would double each probe's round trip)
      if ((it & 15) == 15 &&
          (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || rtc() - t0 > kSpinTicks)) {
        if (lane == 0) __hip_atomic_store(err, 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
  }
  xl = lane < cw ? __builtin_bit_cast(double, v) : 0.0;
  return true;
}

// Swizzled 64 x 64 fp64 tile in LDS: element (i, j) at row i, 16-byte chunk
// (j / 2) ^ (i & 31) -- row-per-lane reads and column-per-lane writes of one
// row are both conflict-free.
__device__ __forceinline__ int swz64(int i, int j) { return i * kBS + ((((j >> 1) ^ (i & 31))) << 1) + (j & 1); }

// T^-1 B for the upper-triangular 64 x 64 T (tT holds T transposed, rdv
// lane k = 1 / T[k][k]), one column of B per lane: column-oriented back
// substitution over all 64 right-hand sides at once.  acc holds the lane's
// column of B on entry, of T^-1 B on exit.  The uniform T values come from
// LDS in 8-value chunks, software-pipelined one chunk ahead (the reads of
// chunk n+1 are issued before the FMAs of chunk n): without it the compiler
// waited on nearly every broadcast read (~15 us per 64 columns).
constexpr int tri_chunks() {
  int c = 0;
  for (int k = kBS - 1; k >= 1; --k) c += (k + 7) / 8;
  return c;
}
constexpr int kTriChunks = tri_chunks();
constexpr int tri_chunk_k(int nth) {
  for (int k = kBS - 1; k >= 1; --k) {
    const int c = (k + 7) / 8;
    if (nth < c) return k;
    nth -= c;
  }
  return 0;
}
constexpr int tri_chunk_i0(int nth) {
  for (int k = kBS - 1; k >= 1; --k) {
    const int c = (k + 7) / 8;
    if (nth < c) return nth * 8;
    nth -= c;
  }
  return 0;
}

__device__ __forceinline__ double lane_value(double v, int k) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  return __builtin_bit_cast(double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(b >> 32), k) << 32) |
                                        (unsigned)__builtin_amdgcn_readlane((int)b, k));
}

template <int N>
__device__ __forceinline__ void tri_read_chunk(const double (*tT)[kBS], double (&c)[8]) {
  constexpr int k = tri_chunk_k(N), i0 = tri_chunk_i0(N);
#pragma unroll
  for (int q = 0; q < 8; q += 2)
    if (i0 + q < k) {
      const double2 t = *reinterpret_cast<const double2*>(&tT[k][i0 + q]);  // T[i][k], T[i+1][k] (uniform)
      c[q] = t.x;
      c[q + 1] = t.y;
    }
}

template <int N>
__device__ __forceinline__ void tri_chunks_from(const double (*tT)[kBS], double rdv, double (&acc)[kBS],
                                                const double (&cur)[8], double xk) {
  if constexpr (N < kTriChunks) {
    constexpr int k = tri_chunk_k(N), i0 = tri_chunk_i0(N);
    double nxt[8];
    if constexpr (N + 1 < kTriChunks) tri_read_chunk<N + 1>(tT, nxt);
    if constexpr (i0 == 0) {  // first chunk of column k: x_k is final
      xk = acc[k] * lane_value(rdv, k);
      acc[k] = xk;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (i0 + q < k) acc[i0 + q] = fma(-cur[q], xk, acc[i0 + q]);
    tri_chunks_from<N + 1>(tT, rdv, acc, nxt, xk);
  }
}

__device__ __forceinline__ void tri_inv_apply(const double (*tT)[kBS], double rdv, double (&acc)[kBS]) {
  double c0[8];
  tri_read_chunk<0>(tT, c0);
  tri_chunks_from<0>(tT, rdv, acc, c0, 0.0);
  acc[0] *= lane_value(rdv, 0);
}

// Bounded wait (LDS spin) until *p >= want or the poller gave up.
// The LDS hand-offs inside a workgroup (xseq -> xs[], done[] -> part[],
// vready -> vb[]) are release stores / acquire loads at workgroup scope: the
// plain LDS data a flag guards is then ordered before the flag store and
// after the flag load (on gfx950 this costs an lgkmcnt wait, no cache work).
__device__ __forceinline__ bool lds_wait(const int* p, int want, const int* abort_flag) {
  if (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= want) return true;
  const unsigned long long t0 = rtc();
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < want) {
    if (__hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0 || rtc() - t0 > kSpinTicks)
      return false;
  }
  return true;
}

constexpr int kRing = 16;  // x vectors in flight between the poller and the compute waves
constexpr int kPf = 4;     // U slices in flight per compute wave
constexpr int kBsThreads = 5 * 64;

template <typename T>
__device__ __forceinline__ void load_slice(double (&us)[16], const T* __restrict__ urow, int c, int n, int w) {
  const int c0 = c * kBS, cw = min(kBS, n - c0);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = 16 * w + q;
    us[q] = (double)dev::load_sel(urow + c0 + min(j, cw - 1), j < cw, T(0));
  }
}

// Row `lane` of a swizzled LDS tile into registers: the 32 reads issued as
// one group (the scheduler otherwise takes them four at a time, one LDS round
// trip per group).
__device__ __forceinline__ void load_tile_row(const double* tile, int lane, double (&m)[kBS]) {
#pragma unroll
  for (int k = 0; k < kBS; k += 2) {
    const double2 v2 = *reinterpret_cast<const double2*>(&tile[swz64(lane, k)]);
    m[k] = v2.x;
    m[k + 1] = v2.y;
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 32, 0);
}

// sum_k m[k] z_k with z broadcast from LDS (uniform ds_read_b128, two values
// per read), 16 reads per group.
__device__ __forceinline__ double row_dot_bcast(const double (&m)[kBS], const double* zv) {
  double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int h = 0; h < kBS; h += 32) {
    double z[32];
#pragma unroll
    for (int k = 0; k < 32; k += 2) {
      const double2 v2 = *reinterpret_cast<const double2*>(&zv[h + k]);
      z[k] = v2.x;
      z[k + 1] = v2.y;
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 1);
#pragma unroll
    for (int k = 0; k < 32; ++k) a[k & 3] = fma(m[h + k], z[k], a[k & 3]);
    __builtin_amdgcn_sched_group_barrier(0x002, 32, 1);
  }
  return (a[0] + a[1]) + (a[2] + a[3]);
}

// One wave solves T v = r, row per lane: the lane's row of T is read from
// T^T in LDS into registers first (64 independent reads), then per step the
// lane-k value is broadcast with v_readlane and the rows above update.
__device__ __forceinline__ double tri_solve_wave(const double (*tT)[kBS], double rdl, double r, int lane) {
  double tr[kBS];
#pragma unroll
  for (int k = 0; k < kBS; ++k) tr[k] = tT[k][lane];
#pragma unroll
  for (int k = kBS - 1; k > 0; --k) {
    const double xl = r * rdl;  // meaningful in lane k
    const uint64_t bb = __builtin_bit_cast(uint64_t, xl);
    const double xk = __builtin_bit_cast(double, ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(bb >> 32), k) << 32) |
                                                     (unsigned)__builtin_amdgcn_readlane((int)bb, k));
    r = lane < k ? fma(-tr[k], xk, r) : r;
  }
  // lane i's r stopped changing at step i: x_i = r_i / T[i][i], no select chain
  return r * rdl;
}

// Block b (64 equations) of the persistent back substitution: 4 compute waves
// + 1 poller wave.  With T = U[b, b], U1 = U[b, b+1], U2 = U[b, b+2]:
//   x_b = T^-1 (y_b - sum_{c >= b+3} U[b, c] x_c) - W2 x_{b+2} - W x_{b+1},
//   W = T^-1 U1, W2 = T^-1 U2 (column back substitutions, backward stable).
// T^-1 itself is never formed: applying an explicit inverse to the running
// right-hand side loses accuracy on ill-conditioned diagonal blocks (the
// zero-pivot rule's U: 2-4x the error of a plain solve), the two W products
// do not (profiles/backsub_r5.txt).
//  prologue (all workgroups at once): T^T, U1, U2 staged in LDS; wave 0 forms
//  W, wave 1 W2;
//  background: the poller polls x_c, c = nb-1 .. b+3, as they land and passes
//  each into an LDS ring; compute wave w accumulates its 16-column slice of
//  U[b, c] x_c from U slices loaded kPf blocks ahead (the poller is the only
//  wave with a global load in flight when it polls, so a poll never waits
//  behind a prefetch -- vmcnt retires loads in order); the poller then solves
//  T v' = y_b - sum (one wave, 64 steps) -- two chain steps before x_b is due;
//  chain: v = v' - W2 x_{b+2} once x_{b+2} lands, x_b = v - W x_{b+1} once
//  x_{b+1} lands (one mat-vec each, the next poll issued before the mat-vec),
//  then x_b is stored sc1: each x value is its own hand-off.
template <typename T>
__global__ __launch_bounds__(kBsThreads) void backsub_persist_kernel(const T* __restrict__ U, int64_t ldu,
                                                                     const T* __restrict__ y, int64_t incy,
                                                                     const int* __restrict__ perm,
                                                                     double* __restrict__ x,
                                                                     double* __restrict__ bnorm, int n,
                                                                     int unit, int* err) {
  __shared__ __attribute__((aligned(16))) double tT[kBS][kBS];  // T^T
  __shared__ __attribute__((aligned(16))) double u1[kBS * kBS];  // U1, then W (swizzled)
  __shared__ __attribute__((aligned(16))) double u2[kBS * kBS];  // U2, then W2 (swizzled)
  __shared__ __attribute__((aligned(16))) double xs[kRing][kBS];
  __shared__ __attribute__((aligned(16))) double zb[2][kBS];  // poller: broadcast vectors
  __shared__ double part[4][kBS];
  __shared__ double rd[kBS];
  __shared__ double ys[kBS];  // y_b: the poller's only global loads are its probes
  __shared__ double vb[kBS];  // wave 0 -> poller: v = v' - W2 x_{b+2}
  __shared__ int xseq, done[4], abort_flag, vready;
  const int b = blockIdx.x, nb = gridDim.x;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int r0 = b * kBS, rows = min(kBS, n - r0);
  const bool has1 = b + 1 < nb, has2 = b + 2 < nb;
  const int c1 = r0 + kBS, cw1 = has1 ? min(kBS, n - c1) : 0;
  const int c2 = r0 + 2 * kBS, cw2 = has2 ? min(kBS, n - c2) : 0;
  const int nbg = nb - b - 3 > 0 ? nb - b - 3 : 0;  // background blocks c = nb-1 .. b+3

  // ---- stage T (transposed, identity-padded), U1, U2 (zero-padded) ---------
  if (t == 0) {
    xseq = 0;
    abort_flag = 0;
    vready = 0;
  }
  if (t < 4) done[t] = 0;
  if (t < 256) {
    const int i = t >> 2, q0 = (t & 3) * 16;  // row i, columns q0 .. q0+15
    const int pr = rowof(perm, r0 + min(i, rows - 1), n);
    if (perm && q0 == 0 && i < rows && perm[r0 + i] != pr)
      __hip_atomic_store(err, 7, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (q0 == 0) ys[i] = i < rows ? (double)y[(int64_t)pr * incy] : 0.0;
    const T* src = U + (int64_t)pr * ldu;
    double tv[16], uv[16], vv[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = q0 + q;
      tv[q] = dev::load_sel(src + r0 + min(j, rows - 1), i < rows && j < rows && j >= i, T(0));
      uv[q] = has1 ? (double)dev::load_sel(src + c1 + min(j, cw1 - 1), i < rows && j < cw1, T(0)) : 0.0;
      vv[q] = has2 ? (double)dev::load_sel(src + c2 + min(j, cw2 - 1), i < rows && j < cw2, T(0)) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int j = q0 + q;
      double d = tv[q];
      if (j == i) {
        d = (i >= rows || unit) ? 1.0 : d;
        rd[i] = 1.0 / d;
        if (bnorm && i < rows) {
          const double yv = (double)y[(int64_t)pr * incy];
          bnorm[r0 + i] = unit ? yv : yv / d;
        }
      }
      tT[j][i] = d;
      u1[i * kBS + j] = uv[q];
      u2[i * kBS + j] = vv[q];
    }
  }
  __syncthreads();
  // ---- wave 0: W = T^-1 U1; wave 1: W2 = T^-1 U2 (one column per lane) -----
  if ((w == 0 && has1) || (w == 1 && has2)) {
    double* m = w == 0 ? u1 : u2;
    double acc[kBS];
#pragma unroll
    for (int i = 0; i < kBS; ++i) acc[i] = m[i * kBS + lane];
    tri_inv_apply(tT, rd[lane], acc);
    // only this wave touches m: overwrite it in place, swizzled
#pragma unroll
    for (int i = 0; i < kBS; ++i) m[swz64(i, lane)] = acc[i];
  }
  __syncthreads();
  const int pr = rowof(perm, r0 + min(lane, rows - 1), n);

  if (w < 4) {
    // ---- compute waves: this wave's 16-column slice of U[b, c] x_c ---------
    const T* urow = U + (int64_t)pr * ldu;
    double us[kPf][16];
#pragma unroll
    for (int d = 0; d < kPf; ++d)
      if (d < nbg) load_slice<T>(us[d], urow, nb - 1 - d, n, w);
    double ra = 0.0, rb = 0.0;
    bool ok = true;
    for (int s0 = 0; s0 < nbg && ok; s0 += kPf) {
#pragma unroll
      for (int d = 0; d < kPf; ++d) {
        const int sq = s0 + d;
        if (sq < nbg && ok) {
          ok = lds_wait(&xseq, sq + 1, &abort_flag);
          if (ok) {
            const double* xv = &xs[sq % kRing][16 * w];
#pragma unroll
            for (int q = 0; q < 16; q += 2) {
              const double2 xx = *reinterpret_cast<const double2*>(xv + q);
              ra = fma(us[d][q], xx.x, ra);
              rb = fma(us[d][q + 1], xx.y, rb);
            }
            if (lane == 0) __hip_atomic_store(&done[w], sq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (sq + kPf < nbg) load_slice<T>(us[d], urow, nb - 1 - (sq + kPf), n, w);
          }
        }
      }
    }
    part[w][lane] = ra + rb;
    if (lane == 0) __hip_atomic_store(&done[w], nbg + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (w != 0) return;
    // ---- wave 0: T v' = y_b - sum, then v = v' - W2 x_{b+2} -----------------
    for (int q = 1; q < 4 && ok; ++q) ok = lds_wait(&done[q], nbg + 1, &abort_flag);
    if (!ok) return;
    const double r = ys[lane] - ((part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]));
    double v = tri_solve_wave(tT, rd[lane], r, lane);
    if (has2) {
      double m[kBS];
      load_tile_row(u2, lane, m);
      if (!lds_wait(&xseq, nbg + 1, &abort_flag)) return;  // x_{b+2}: the ring's last entry
      v -= row_dot_bcast(m, xs[nbg % kRing]);
    }
    vb[lane] = v;
    if (lane == 0) __hip_atomic_store(&vready, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }

  // ---- poller wave: x_c, c = nb-1 .. b+2, into the ring; then the chain ----
  double wrow[kBS];  // row `lane` of W
  if (has1) load_tile_row(u1, lane, wrow);
  bool ok = true;
  const int nring = has2 ? nbg + 1 : 0;
  for (int sq = 0; sq < nring && ok; ++sq) {
    const int c = nb - 1 - sq;
    if (sq >= kRing) {  // the ring slot is free once every compute wave used x of sq - kRing
      const int need = sq - kRing + 1;
      for (int q = 0; q < 4 && ok; ++q) ok = lds_wait(&done[q], need, &abort_flag);
    }
    double xl = 0.0;
    ok = ok && poll_x(x, c * kBS, min(kBS, n - c * kBS), err, false, xl);
    if (ok) {
      xs[sq % kRing][lane] = xl;
      if (lane == 0) __hip_atomic_store(&xseq, sq + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  double xl1 = 0.0;
  if (has1 && ok) ok = poll_x(x, c1, cw1, err, false, xl1);
  if (ok) ok = lds_wait(&vready, 1, &abort_flag);
  if (!ok) {
    // x_b is never written: make sure the host hears of it even when no
    // other workgroup is left to time out on it (block 0)
    if (lane == 0) {
      __hip_atomic_store(&abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      int zero = 0;
      __hip_atomic_compare_exchange_strong(err, &zero, 3, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  double v = vb[lane];
  if (has1) {
    zb[1][lane] = xl1;
    v -= row_dot_bcast(wrow, zb[1]);
  }
  if (lane < rows)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(x + r0 + lane), __builtin_bit_cast(unsigned long long, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- fallback: one launch per block ----------------------------------------

template <typename T>
__global__ __launch_bounds__(64) void diag_solve_kernel(const T* __restrict__ U, int64_t ldu,
                                                        const int* __restrict__ perm,
                                                        double* __restrict__ yw,
                                                        double* __restrict__ x, int i0, int nb,
                                                        int unit, int n) {
  double row[kBS];
  double rinv;
  load_diag<T>(U, ldu, perm, n, i0, nb, unit, row, rinv);
  const int l = threadIdx.x & 63;
  const double xv = solve_diag(row, rinv, dev::load_sel(yw + i0 + min(l, nb - 1), l < nb), nb);
  if (l < nb) x[i0 + l] = xv;
}

// Every workgroup subtracts block [i0, i0+nb)'s solved x from its rows above
// (wave per row); workgroup 0 owns the 64 rows right above the block and,
// once they are final, solves that diagonal block too.
template <typename T>
__global__ __launch_bounds__(256) void backsub_step_kernel(const T* __restrict__ U, int64_t ldu,
                                                           const int* __restrict__ perm,
                                                           double* __restrict__ yw,
                                                           double* __restrict__ x, int i0, int nb,
                                                           int unit, int n) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int p0 = i0 > kBS ? i0 - kBS : 0;  // the next diagonal block [p0, i0)
  const double xl = dev::load_sel(x + i0 + min(lane, nb - 1), lane < nb);
  if (blockIdx.x == 0) {
    constexpr int kRows = kBS / 4;
    double v[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      v[k] = dev::load_sel(U + (int64_t)rowof(perm, min(r, i0 - 1), n) * ldu + i0 + min(lane, nb - 1),
                           lane < nb && r < i0) * xl;
    }
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int r = p0 + wv * kRows + k;
      const double sum = dev::wave_sum(v[k]);
      if (lane == 0 && r < i0) yw[r] -= sum;
    }
    __syncthreads();
    if (wv == 0) {
      double row[kBS];
      double rinv;
      load_diag<T>(U, ldu, perm, n, p0, i0 - p0, unit, row, rinv);
      const int l = lane;
      const double xv = solve_diag(row, rinv, dev::load_sel(yw + p0 + min(l, i0 - p0 - 1), l < i0 - p0), i0 - p0);
      if (l < i0 - p0) x[p0 + l] = xv;
    }
    return;
  }
  const int nw = (gridDim.x - 1) * 4;
  for (int r = (blockIdx.x - 1) * 4 + wv; r < p0; r += nw) {
    double v = dev::load_sel(U + (int64_t)rowof(perm, r, n) * ldu + i0 + min(lane, nb - 1), lane < nb) * xl;
    v = dev::wave_sum(v);
    if (lane == 0) yw[r] -= v;
  }
}

template <typename T>
int backsub_impl(const T* U, int64_t ldu, const T* y, int64_t incy, double* x, double* bnorm,
                 int64_t n, int unit, double* yw, hipStream_t s, const int* perm, int* err, bool x_ready) {
  const int64_t nblk = (n + kBS - 1) / kBS;
  // the persistent form needs every block resident (flag hand-offs);
  // checked once per (type, block count)
  bool persist = nblk <= kMaxPersistBlocks;
  if (persist) {
    int per = 0;
    persist = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, backsub_persist_kernel<T>, kBsThreads, 0) == hipSuccess &&
              coresident(per, nblk);
  }
  if (persist) {
    // the error word lives in yw when the caller has none (zeroed here); a
    // caller's word is the caller's to clear: it may already carry an
    // upstream code (resident LU abort, row map), which stops this kernel
    // at its first poll and must reach the host
    int* e = err ? err : reinterpret_cast<int*>(yw);
    if (x_ready && !err) return GELIM_FAIL(GELIM_E_ARG, "backsub: a prefilled x needs the caller's error word");
    if (!x_ready) {
      hipLaunchKernelGGL(fill_sent_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                         reinterpret_cast<uint64_t*>(x), (int)n, err ? nullptr : e);
      HIP_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(backsub_persist_kernel<T>, dim3((unsigned)nblk), dim3(kBsThreads), 0, s, U, ldu, y, incy,
                       perm, x, bnorm, (int)n, unit, e);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  hipLaunchKernelGGL(copy_y_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, U, ldu, y, incy,
                     perm, yw, bnorm, (int)n, unit);
  HIP_TRY(hipGetLastError());
  int64_t i0 = (n - 1) / kBS * kBS;
  hipLaunchKernelGGL(diag_solve_kernel<T>, dim3(1), dim3(64), 0, s, U, ldu, perm, yw, x, (int)i0,
                     (int)(n - i0), unit, (int)n);
  HIP_TRY(hipGetLastError());
  for (int64_t i1 = n; i0 > 0; i1 = i0, i0 -= kBS) {
    const int nb = (int)(i1 - i0);
    const int64_t rows = i0 > kBS ? i0 - kBS : 0;  // rows above the next block
    const int blocks = 1 + (int)std::min<int64_t>((rows + 3) / 4, 1024);
    hipLaunchKernelGGL(backsub_step_kernel<T>, dim3(blocks), dim3(256), 0, s, U, ldu, perm, yw, x,
                       (int)i0, nb, unit, (int)n);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

}  // namespace

int backsub_f64(const double* U, int64_t ldu, const double* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s, const int* perm,
                int* err, bool x_ready) {
  return backsub_impl<double>(U, ldu, y, incy, x, bnorm, n, unit, yw, s, perm, err, x_ready);
}

unsigned backsub_sentinel_word() { return (unsigned)(kXSent & 0xffffffffu); }

int backsub_f32(const float* U, int64_t ldu, const float* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s, const int* perm,
                int* err) {
  return backsub_impl<float>(U, ldu, y, incy, x, bnorm, n, unit, yw, s, perm, err, false);
}

}  // namespace gelim

extern "C" int gelim_gpu_backsub(const double* dU, int64_t ldu, const double* dy, int64_t incy,
                                 double* dx, double* dbnorm, int64_t n, int unit, void* stream) {
  if (n <= 0) return GELIM_FAIL(GELIM_E_ARG, "backsub: n <= 0");
  hipStream_t s = (hipStream_t)stream;
  double* yw = nullptr;
  HIP_TRY(hipMallocAsync((void**)&yw, sizeof(double) * (n + 2), s));
  int rc = gelim::backsub_f64(dU, ldu, dy, incy, dx, dbnorm, n, unit, yw, s, nullptr, nullptr, false);
  HIP_TRY(hipFreeAsync(yw, s));
  return rc;
}
