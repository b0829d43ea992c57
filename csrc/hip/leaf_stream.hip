// Streamed 32-column leaf: the m x 32 panel factorisation of the wide-panel
// LU (biglu.hip) for panels taller than the register-resident leaf holds
// (leaf.h: 256 participants x 4 waves x 256 rows = 262144 rows, the whole
// register file of the chip).  The distributed solver's owner factors its
// panel over ALL remaining rows, so at n ~ 537k (8 x 288 GB of fp64 slabs,
// SURVEY §5.7; the reference sizes its MPI buffers by n/(P-1),
// OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:218) the first panels have
// more rows than any register leaf.
//
// What it computes: exactly what the register leaf computes, bit for bit --
// the same pivot rule (largest key, ties to the lowest leaf row; the ZERO
// rule's position keys), the same reciprocal (v_rcp + two Newton steps), the
// same FMA per element in the same order, logical pivoting with the LAPACK
// interchange replay (ipiv, the net row movement in `pairs`, rows written to
// their final positions at the end).  tests/test_gpu_biglu.py compares the
// two leaves bitwise at m <= 262144 (GELIM_LEAF_STREAM=1) and this one with
// LAPACK-order pivots of torch.linalg.lu_factor above it.
//
// How: the panel stays in HBM and every column is two stream-ordered
// launches (no cross-workgroup hand-off, so nothing needs co-residency and
// the lookahead GEMMs beside it cannot starve it):
//  * sweep(J): every live row gets the pending pivot J-1 (its multiplier
//    into column J-1, the rank-1 update of columns J..31) and offers its
//    column-J key; a half-wave owns one row at a time, lane c its column c,
//    so each row is ONE coalesced 256-byte access and only the 128-byte
//    lines holding live columns move; per-workgroup winners go to a small
//    candidate array;
//  * pick(J): one wave merges the candidates, reads the pivot row, takes
//    1/pivot, replays the interchange (a <= 64-entry table in its lanes) and
//    records ipiv.
// Per column the sweep moves ~m x (32 - J) x 16 bytes: ~0.25 ms of HBM time
// per 32 columns at m = 300000, against ~600 s of trailing GEMMs at n = 537k.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace big {
namespace sleaf {
namespace {

constexpr int LW = 32;       // leaf width (leaf.h)
constexpr int NT = 256;      // sweep workgroup: 4 waves, 8 rows per pass
constexpr int kMaxG = 1024;  // sweep workgroups (candidate slots)

// Device scratch of one streamed leaf (after the register leaf's exchange
// areas in the leaf workspace; nothing in it needs zeroing).
struct Scratch {
  unsigned long long ckey[kMaxG];  // per sweep workgroup: best key of the column
  unsigned crow[kMaxG];            //   ... and its leaf row (lowest on ties)
  double u[LW];                    // pivot row of the last picked column
  double rinv;                     // its 1 / pivot (0 for a zero pivot)
  int piv[LW];                     // leaf row picked at each column
  int tcnt;                        // interchange table: entries in use
  int trow[2 * LW], tpos[2 * LW];  // displaced row trow[e] now sits at position tpos[e]
};

struct Args {
  double* A;  // leaf top-left (row c0, column c0 of the system)
  int64_t lda;
  int m, col0;
  int* ipiv;
  int* pairs;
  int* info;
  Scratch* sc;
};

__device__ __forceinline__ unsigned lo32(double x) { return (unsigned)__double_as_longlong(x); }
__device__ __forceinline__ unsigned hi32(double x) { return (unsigned)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ double mkd(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// the register leaf's reciprocal (leaf.h recip): v_rcp_f64 + two Newton steps
__device__ __forceinline__ double recip(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  return fma(r, fma(-p, r, 1.0), r);
}

// (key, row) merge: larger key wins, the lower row on equal non-zero keys
__device__ __forceinline__ bool better(unsigned long long k1, unsigned r1, unsigned long long k0, unsigned r0) {
  return k1 > k0 || (k1 == k0 && k1 != 0 && r1 < r0);
}

// wave arg-max of (key, row): largest key, lowest row; result uniform
__device__ __forceinline__ void wave_best(unsigned long long& k, unsigned& r) {
  const unsigned long long km = dev::wave_max_u64(k);
  const unsigned rm = dev::wave_min_u32(k == km ? r : 0xffffffffu);
  k = km;
  r = rm;
}

// position of leaf row r after the interchanges so far (ZERO rule keys)
__device__ __forceinline__ int position(int r, const int* trow, const int* tpos, int cnt) {
  int p = r;
  for (int e = 0; e < cnt; ++e) p = trow[e] == r ? tpos[e] : p;
  return p;
}

// sweep(J), J = 0..LW: pending pivot J-1 applied to every live row, then
// (J < LW) the column-J candidates.  Half-wave h of wave w handles rows
// (blockIdx * 8 + 2 w + h) + 8 G k.
template <int MODE>
__global__ __launch_bounds__(NT) void sweep_kernel(Args g, int J) {
  __shared__ int spiv[LW];
  __shared__ int strow[2 * LW], stpos[2 * LW];
  __shared__ double su[LW];
  __shared__ unsigned long long wk[NT / 64];
  __shared__ unsigned wr[NT / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, h = lane >> 5, c = lane & 31;
  Scratch* sc = g.sc;
  if (t < J) spiv[t] = sc->piv[t];
  if (t < LW) su[t] = J > 0 ? sc->u[t] : 0.0;
  const int cnt = MODE == 0 ? sc->tcnt : 0;
  if (MODE == 0 && t < cnt) {
    strow[t] = sc->trow[t];
    stpos[t] = sc->tpos[t];
  }
  const double rinv = J > 0 ? sc->rinv : 0.0;
  __syncthreads();
  const int c_lo = J > 0 ? J - 1 : 0;  // first column read / written
  unsigned long long bk = 0;
  unsigned br = 0xffffffffu;
  const int64_t stride = (int64_t)gridDim.x * (NT / 32);
  for (int64_t r = (int64_t)blockIdx.x * (NT / 32) + 2 * wave + h; r < g.m; r += stride) {
    bool live = true;
    for (int k = 0; k < J; ++k) live = live && spiv[k] != (int)r;
    double* row = g.A + r * g.lda;
    double x = c >= c_lo ? row[c] : 0.0;
    if (J > 0 && live) {
      // this row's multiplier of pivot J-1 (lane J-1 of the half), then the
      // rank-1 update of columns J.. -- the register leaf's FMAs
      const int src = (lane & 32) + J - 1;
      const double xm = mkd((unsigned)__shfl((int)lo32(x), src), (unsigned)__shfl((int)hi32(x), src));
      const double l = xm * rinv;
      if (c == J - 1) x = l;
      else if (c >= J) x = fma(-l, su[c], x);
      if (c >= c_lo) row[c] = x;
    }
    if (J < LW) {
      const int src = (lane & 32) + J;
      const double v = mkd((unsigned)__shfl((int)lo32(x), src), (unsigned)__shfl((int)hi32(x), src));
      unsigned long long k;
      if constexpr (MODE == 1) {
        k = dev::pivot_ukey_t<1>(v, false, live);
      } else {
        const int p = position((int)r, strow, stpos, cnt);
        k = dev::pivot_ukey_t<0>(v, p == J, live);
        k = k == 0 ? 0 : (k << 32) | (0xffffffffu - (unsigned)p);
      }
      if (better(k, (unsigned)r, bk, br)) {
        bk = k;
        br = (unsigned)r;
      }
    }
  }
  if (J == LW) return;
  wave_best(bk, br);
  if (lane == 0) {
    wk[wave] = bk;
    wr[wave] = br;
  }
  __syncthreads();
  if (t == 0) {
    unsigned long long k = wk[0];
    unsigned r = wr[0];
    for (int w = 1; w < NT / 64; ++w)
      if (better(wk[w], wr[w], k, r)) {
        k = wk[w];
        r = wr[w];
      }
    sc->ckey[blockIdx.x] = k;
    sc->crow[blockIdx.x] = r;
  }
}

// pick(J): one wave.  The global winner, its row (pivot J-1 already applied
// by sweep(J)), 1/pivot, the interchange replay (leaf.h table_swap) and ipiv.
__global__ __launch_bounds__(64) void pick_kernel(Args g, int J, int G) {
  const int lane = threadIdx.x;
  Scratch* sc = g.sc;
  unsigned long long bk = 0;
  unsigned br = 0xffffffffu;
  for (int p = lane; p < G; p += 64)
    if (better(sc->ckey[p], sc->crow[p], bk, br)) {
      bk = sc->ckey[p];
      br = sc->crow[p];
    }
  wave_best(bk, br);
  // every live row has a non-zero key and m >= LW rows, so a row always wins
  const int pr = (int)br;
  if (bk == 0 || pr < 0 || pr >= g.m) {  // broken invariant: report (code 10), never index through it
    if (lane == 0) g.info[1] = 10;
    return;
  }
  const double* prow = g.A + (int64_t)pr * g.lda;
  const double uc = lane < LW ? prow[lane] : 0.0;
  const double pv = prow[J];
  const bool zero = !(pv != 0.0);
  if (lane < LW) sc->u[lane] = uc;
  if (lane == 0) {
    sc->rinv = zero ? 0.0 : recip(pv);
    sc->piv[J] = pr;
    if (zero && g.info[0] == 0) atomicCAS(g.info, 0, g.col0 + J + 1);
  }
  // interchange replay: pr moves to position J, the row at J to pr's spot q
  int cnt = J == 0 ? 0 : sc->tcnt;
  int trow = lane < cnt ? sc->trow[lane] : -1, tpos = lane < cnt ? sc->tpos[lane] : -1;
  const uint64_t m1 = __ballot(lane < cnt && trow == pr);
  const int q = m1 ? __builtin_amdgcn_readlane(tpos, __ffsll((long long)m1) - 1) : pr;
  if (q != J) {
    const uint64_t m2 = __ballot(lane < cnt && tpos == J);
    const int rj = m2 ? __builtin_amdgcn_readlane(trow, __ffsll((long long)m2) - 1) : J;
    const int e1 = m1 ? __ffsll((long long)m1) - 1 : cnt++;
    const int e2 = m2 ? __ffsll((long long)m2) - 1 : cnt++;
    if (lane == e1) {
      trow = pr;
      tpos = J;
    }
    if (lane == e2) {
      trow = rj;
      tpos = q;
    }
  }
  if (lane < cnt) {
    sc->trow[lane] = trow;
    sc->tpos[lane] = tpos;
  }
  if (lane == 0) {
    sc->tcnt = cnt;
    g.ipiv[g.col0 + J] = g.col0 + q;
  }
}

// the net row movement: pairs (count, then (dst, src) leaf rows) and every
// displaced row written to its final position (through LDS: a permutation)
__global__ __launch_bounds__(256) void finish_kernel(Args g) {
  __shared__ double rows[2 * LW][LW];
  __shared__ int dst[2 * LW];
  const int t = threadIdx.x;
  const Scratch* sc = g.sc;
  const int cnt = sc->tcnt;
  for (int i = t; i < cnt * LW; i += 256) {
    const int e = i / LW, c = i % LW;
    rows[e][c] = g.A[(int64_t)sc->trow[e] * g.lda + c];
  }
  if (t < cnt) {
    dst[t] = sc->tpos[t];
    g.pairs[1 + 2 * t] = sc->tpos[t];
    g.pairs[2 + 2 * t] = sc->trow[t];
  }
  if (t == 0) g.pairs[0] = cnt;
  __syncthreads();
  for (int i = t; i < cnt * LW; i += 256) {
    const int e = i / LW, c = i % LW;
    g.A[(int64_t)dst[e] * g.lda + c] = rows[e][c];
  }
}

}  // namespace

size_t scratch_bytes() { return (sizeof(Scratch) + 255) & ~size_t(255); }

int sweep_grid(int64_t m) { return (int)std::min<int64_t>(kMaxG, std::max<int64_t>(1, (m + 63) / 64)); }

// Factor the m x 32 leaf at A (row / column c0 of the system) in place; the
// outputs and their format are the register leaf's (biglu.hip leaf_factor).
int factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
           void* scratch, hipStream_t s) {
  if (m < LW || m > 0x7fffffff) return GELIM_FAIL(GELIM_E_ARG, "streamed leaf: m out of range");
  Args a{A, lda, (int)m, (int)c0, ipiv, pairs, info, static_cast<Scratch*>(scratch)};
  const int G = sweep_grid(m);
  for (int J = 0; J <= LW; ++J) {
    if (mode == GELIM_PIVOT_PARTIAL)
      hipLaunchKernelGGL(sweep_kernel<1>, dim3((unsigned)G), dim3(NT), 0, s, a, J);
    else
      hipLaunchKernelGGL(sweep_kernel<0>, dim3((unsigned)G), dim3(NT), 0, s, a, J);
    if (J < LW) hipLaunchKernelGGL(pick_kernel, dim3(1), dim3(64), 0, s, a, J, G);
  }
  hipLaunchKernelGGL(finish_kernel, dim3(1), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace sleaf
}  // namespace big
}  // namespace gelim
