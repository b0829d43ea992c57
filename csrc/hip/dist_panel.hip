// Native per-block steps of the distributed Gauss solver
// (parallel/dist_gauss.py): the owner's factorisation of one outer panel
// and every rank's application of a broadcast panel to its own columns.
//
// What it replaces: the reference's MPI master/worker elimination
// (OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:124-255), where rank 0
// ships whole rows to the workers and back at every pivot.  Here the matrix
// is column block-cyclic (blocks of D columns, D a multiple of the 32-column
// leaf) and resident: the owner factors its m x D panel with the wide-panel
// engine's multi-workgroup leaves (biglu.hip) and broadcasts
// [panel | leaf pair lists] once; every rank then applies it to its trailing
// columns -- the leaves' row movement in one launch, U12 = L11^-1 A12 by
// 32-row blocks, and the trailing update as one K = D fp64 MFMA GEMM
// (dgemm.hip).  Each call issues the whole launch sequence from C++ on the
// caller's stream (one ctypes crossing per block step instead of dozens).
//
// Storage: a rank's slab holds ALL n rows of its local columns, row-major
// (row 0 = global row 0), leading dimension ld; local column c of the slab is
// some global column, the pair lists use global row numbers relative to each
// leaf's diagonal.  n must be a multiple of 32 (dist_gauss.py pads the system
// with an identity block).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "gelim/internal.h"

namespace gelim {
int dgemm(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
          int64_t N, int64_t K, double alpha, hipStream_t s);
int dgemm_capped(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate = 1);
namespace big {
int leaf_width();
int leaf_factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
                void* ws, int set, hipStream_t s, unsigned long long* stamps = nullptr);
int laswp_trsm(double* A, int64_t lda, int64_t c0, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
               int64_t trsm_end, int64_t nrows, const int* pairs, hipStream_t s, const double* L, int64_t ldl);
int laswp_panel(double* A, int64_t lda, int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot,
                int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, hipStream_t s, int max_wg = 0);
int panel_trsm(double* C, int64_t ldc, int64_t ncols, int64_t nb, const double* L, int64_t ldl, hipStream_t s,
               int max_wg = 0);
bool trsm_fused();
int leaf_cus(int64_t m);
int compose_pairs(int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot, int* net, hipStream_t s);
int laswp_net_max();
int64_t compose_max_rows();
int laswp_net(double* A, int64_t lda, const int* net, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
              hipStream_t s, int max_wg);
}  // namespace big
}  // namespace gelim

namespace {
constexpr int64_t kLW = 32;
constexpr int64_t kSlot = 1 + 4 * 32 + 3;  // ints per leaf pair list (plan.hip's kBigPairSlot)
}  // namespace

extern "C" int64_t gelim_dist_pair_slot(void) { return kSlot; }

// Ints of a panel's composed row movement: [valid, count, (dst, src) x
// laswp_net_max()] -- valid = 0 when the panel is too tall for the LDS row
// map of the composition (the pair lists are replayed instead).
extern "C" int64_t gelim_dist_net_ints(void) { return 2 + 2 * (int64_t)gelim::big::laswp_net_max(); }

namespace {
__global__ void set_word_kernel(int* p, int v) {
  if (threadIdx.x == 0) *p = v;
}
}  // namespace

// The panel's leaf pair lists (nleaves lists at pairs, kSlot ints apart)
// composed into ONE permutation of <= 64 rows per leaf (net: see
// gelim_dist_net_ints), or net[0] = 0 when the panel's m rows exceed the
// composition's LDS map: then every apply replays the lists instead.
// Returns 1 when composed, 0 when not (decided on the host from n - k and
// nleaves, so callers know without a device read), < 0 on errors.
extern "C" int gelim_dist_panel_compose(int64_t n, int64_t k, int nleaves, const int32_t* pairs, int32_t* net,
                                        void* stream) {
  using namespace gelim;
  hipStream_t s = (hipStream_t)stream;
  const bool ok = n - k <= big::compose_max_rows() && nleaves * 2 * kLW <= big::laswp_net_max();
  if (ok) GELIM_TRY(big::compose_pairs(n, k, nleaves, pairs, kSlot, net + 1, s));
  hipLaunchKernelGGL(set_word_kernel, dim3(1), dim3(64), 0, s, net, ok ? 1 : 0);
  HIP_TRY(hipGetLastError());
  return ok ? 1 : 0;
}

// Factor rows [k, n) x local columns [lc, lc + wg) of the slab A in place
// (wg a multiple of 32).  Leaf l's pivots go to ipiv[k + 32 l + J] (global
// rows), its net row movement to pairs + l * slot; info[0] = 1 + the first
// zero-pivot column (global).  ws: the leaf exchange workspace, zeroed before
// the first leaf of a solve; leaf0: the solve's running leaf counter.
// upd_end > lc + wg: every leaf also updates local columns [lc + wg, upd_end)
// -- the next block when this rank factors it next (one rank: plan.hip's
// lookahead form, so that block is up to date the moment this panel is) --
// after waiting, once leaf 0 is factored, for wait_ev (may be null): the
// event after which those columns carry every earlier panel.
extern "C" int gelim_dist_panel_factor(double* A, int64_t lda, int64_t n, int64_t k, int64_t lc, int64_t wg,
                                       int pivot, int32_t* ipiv, int32_t* pairs, int32_t* info, void* ws, int leaf0,
                                       int64_t upd_end, void* wait_ev, void* stream) {
  using namespace gelim;
  hipStream_t s = (hipStream_t)stream;
  if (wg <= 0 || wg % kLW || n % kLW || k + wg > n || (lc & 1) || (lda & 1))
    return GELIM_FAIL(GELIM_E_ARG, "dist_panel_factor: widths must be multiples of 32 (even offsets)");
  const int64_t ue = std::max(upd_end, lc + wg);
  for (int64_t l = 0; l * kLW < wg; ++l) {
    const int64_t c0 = k + l * kLW, col = lc + l * kLW;
    int* pr = pairs + l * kSlot;
    GELIM_TRY(big::leaf_factor(A + c0 * lda + col, lda, n - c0, c0, pivot, ipiv, pr, info, ws, leaf0 + (int)l, s));
    if (l == 0 && wait_ev != nullptr && ue > lc + wg) HIP_TRY(hipStreamWaitEvent(s, (hipEvent_t)wait_ev, 0));
    // the leaf's row movement on the panel's other columns (and the next
    // block's), TRSM of its U rows on the columns right of it
    GELIM_TRY(big::laswp_trsm(A + c0 * lda, lda, col, lc, col, col + kLW, ue, ue, n - c0, pr, s, nullptr, 0));
    const int64_t c1 = col + kLW, r1 = c0 + kLW;
    if (c1 < ue && r1 < n)
      GELIM_TRY(dgemm(A + r1 * lda + c1, lda, A + r1 * lda + col, lda, A + c0 * lda + c1, lda, n - r1, ue - c1, kLW,
                      -1.0, s));
  }
  return GELIM_OK;
}

// Apply a factored panel (its rows [k, n) as a row-major (n - k) x wg block L
// with leading dimension ldl, and its leaf pair lists) to local columns
// [cb, ce) of the slab C: the leaves' row movement, U12 = L11^-1 A12 on rows
// [k, k + wg), A22 -= L21 U12 on rows [k + wg, n).  net (may be null): the
// panel's composed movement (gelim_dist_panel_compose); when valid it is
// applied as one gather/scatter instead of replaying the lists per column
// (~90 us a call, round-3 trace).  max_wg > 0: every launch on at most
// max_wg CUs (the lookahead side stream, which must leave the leaves of the
// concurrent panel factorisation free CUs; plan.hip's cap).
extern "C" int gelim_dist_panel_apply(double* C, int64_t ldc, int64_t n, int64_t k, int64_t cb, int64_t ce,
                                      const double* L, int64_t ldl, int64_t wg, const int32_t* pairs,
                                      const int32_t* net, int net_valid, int max_wg, void* stream) {
  using namespace gelim;
  hipStream_t s = (hipStream_t)stream;
  if (ce <= cb) return GELIM_OK;
  if (wg <= 0 || wg % kLW || n % kLW || k + wg > n || (cb & 1) || (ldc & 1) || (ldl & 1))
    return GELIM_FAIL(GELIM_E_ARG, "dist_panel_apply: widths must be multiples of 32 (even offsets)");
  const int nl = (int)(wg / kLW);
  if (net != nullptr && net_valid)
    GELIM_TRY(big::laswp_net(C + k * ldc, ldc, net + 1, 0, 0, cb, ce, s, max_wg));
  else
    GELIM_TRY(big::laswp_panel(C, ldc, n, k, nl, pairs, kSlot, 0, 0, cb, ce, s, max_wg));
  if (big::trsm_fused() && wg <= 256) {
    GELIM_TRY(big::panel_trsm(C + k * ldc + cb, ldc, ce - cb, wg, L, ldl, s, max_wg));
  } else {
    for (int64_t j = 0; j < nl; ++j) {
      const int64_t r = k + j * kLW;
      GELIM_TRY(big::laswp_trsm(C + r * ldc, ldc, 0, 0, 0, cb, ce, ce, n - r, nullptr, s,
                                L + (j * kLW) * ldl + j * kLW, ldl));
      if (j + 1 < nl)
        GELIM_TRY(dgemm(C + (r + kLW) * ldc + cb, ldc, L + ((j + 1) * kLW) * ldl + j * kLW, ldl, C + r * ldc + cb,
                        ldc, wg - (j + 1) * kLW, ce - cb, kLW, -1.0, s));
    }
  }
  if (k + wg < n)
    GELIM_TRY(dgemm_capped(C + (k + wg) * ldc + cb, ldc, L + wg * ldl, ldl, C + k * ldc + cb, ldc, n - k - wg, ce - cb,
                           wg, -1.0, max_wg, s));
  return GELIM_OK;
}

// CUs the side stream may use beside the leaves of an m-row panel: the CU
// count less max(64, the CUs the largest leaf needs + 8) (plan.hip's rule)
extern "C" int gelim_dist_side_cap(int64_t m) {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int reserve = std::max(64, gelim::big::leaf_cus(m) + 8);
  return ncu > reserve + 8 ? ncu - reserve : std::max(8, ncu / 2);
}
