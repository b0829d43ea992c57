// Gauss solver plan: owns the device working system and orchestrates the
// kernels of one solve, captured once into a hipGraph and replayed.
//
// Why a graph: the per-pivot algorithm is 2n dependent launches and the
// blocked one ~3n/w; issued eagerly each launch costs ~3-4 us of host time
// (MI355X_MICROARCH.md price list, graph-replay-floor), so the solve would be
// host-bound.  Captured, each boundary costs ~1.5 us on the device only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "gelim/internal.h"

namespace gelim {
int64_t panel_width_for(int64_t m);
int panel_factor(double* P, int64_t ldp, int64_t m, int64_t w, int64_t row0, int mode, int* piv,
                 int* info, hipStream_t s, int* pairs);
int64_t lu_panel_buffer_ld(int64_t n);
int lu_step(double* A, int64_t lda, int64_t n, int64_t kp, int64_t wp, const int* pairs_prev,
            int64_t k, int64_t w, int mode, int* piv, int* info, int* pairs, hipStream_t s,
            const double* buf, double* lout, const double* lprev, int64_t ldL, unsigned* nflags = nullptr,
            double* nbuf = nullptr, int64_t nk = 0, int64_t nw = 0);
int lu_narrow(double* A, int64_t lda, int64_t n, int64_t kp, int64_t wp, const int* pairs,
              int64_t k, int64_t w, double* buf, hipStream_t s, const double* L, int64_t ldL);
int pairs_trsm(double* C, int64_t ldc, int64_t ncols, const double* L, int64_t ldl, int64_t w,
               const int* pairs, hipStream_t s);
int swap_trsm(double* C, int64_t ldc, int64_t ncols, const double* L, int64_t ldl, int64_t w,
              const int* piv, double* tmp, hipStream_t s);
int gemm_update(double* C, int64_t ldc, const double* L, int64_t ldl, const double* U,
                int64_t ldu, int64_t M, int64_t N, int64_t K, hipStream_t s);
// x_ready: x already holds the hand-off sentinel (backsub_sentinel_word() in
// both halves of every value) and err is the caller's, cleared by the caller
int backsub_f64(const double* U, int64_t ldu, const double* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s,
                const int* perm = nullptr, int* err = nullptr, bool x_ready = false);
unsigned backsub_sentinel_word();
int backsub_f32(const float* U, int64_t ldu, const float* y, int64_t incy, double* x,
                double* bnorm, int64_t n, int unit, double* yw, hipStream_t s,
                const int* perm = nullptr, int* err = nullptr);
int dgemm(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
          int64_t N, int64_t K, double alpha, hipStream_t s);
int dgemm_capped(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate = 1);
namespace big {
size_t workspace_bytes();
int leaf_width();
int64_t max_rows();
int64_t compose_max_rows();
int leaf_cus(int64_t m);
int leaf_factor(double* A, int64_t lda, int64_t m, int64_t c0, int mode, int* ipiv, int* pairs, int* info,
                void* ws, int set, hipStream_t s, unsigned long long* stamps = nullptr);
int laswp_trsm(double* A, int64_t lda, int64_t c0, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
               int64_t trsm_end, int64_t nrows, const int* pairs, hipStream_t s, const double* L = nullptr,
               int64_t ldl = 0);
int laswp_panel(double* A, int64_t lda, int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot,
                int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, hipStream_t s, int max_wg = 0);
int panel_trsm(double* C, int64_t ldc, int64_t ncols, int64_t nb, const double* L, int64_t ldl, hipStream_t s,
               int max_wg = 0);
int compose_pairs(int64_t n, int64_t c0, int nleaves, const int* pairs, int64_t slot, int* net, hipStream_t s);
int laswp_net_max();
int laswp_net(double* A, int64_t lda, const int* net, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend,
              hipStream_t s, int max_wg);
bool trsm_fused();
int tail_gemv(const double* A, int64_t lda, int64_t n, int64_t K, const double* x, double* y, double* bnorm,
              hipStream_t s);
int fold_info(int* info, const int* tinfo, int64_t K, hipStream_t s);
}  // namespace big
int64_t rlu_max_n();
bool rlu_coresident(int64_t n);
size_t rlu_workspace_bytes(int64_t n);
int rlu_factor(const double* src, int64_t lds, double* work, int64_t ldw, int64_t n, int mode,
               int* piv, int* info, void* ws, hipStream_t s, unsigned long long* stamps = nullptr,
               bool flags_ready = false);
// the hand-off flag words rlu_factor clears before its launch (a caller that
// clears them in its own prologue passes flags_ready)
WordFill rlu_flags_fill(int64_t n, void* ws);
template <typename T>
int pivot_elimination(T* A, int64_t lda, int64_t n, int mode, T* mcol, int* info, hipStream_t s, int* ipiv,
                      double* diag);
template <typename T>
int pivot_persistent(T* A, int64_t lda, int64_t n, int mode, int* info, int* ipiv, double* diag, void* ws,
                     hipStream_t s);
size_t pivot_persist_ws_bytes(int64_t n);
template <typename T>
int pivot_lower_resolve(const T* A, int64_t lda, int64_t n, const int* ipiv, const double* diag, const double* c,
                        T* y, hipStream_t s);
}  // namespace gelim

struct gelim_gauss_plan {
  int64_t n = 0, lda = 0;
  int algo = 0, pivot = 0, eb = 8;
  bool use_graph = true;
  void* work = nullptr;
  int* piv = nullptr;
  int* info = nullptr;
  double* yw = nullptr;
  void* mcol = nullptr;
  double* diag = nullptr;                // hip-pivot: pivot values of the stored factors
  void* ry = nullptr;                    // hip-pivot re-solve: L~^-1 P c (plan dtype)
  double* tmp = nullptr;
  void* pws = nullptr;                   // hip-pivot: the persistent kernel's exchange granules
  hipStream_t cap = nullptr;
  hipStream_t side = nullptr;            // lookahead: wide trailing updates
  std::vector<hipEvent_t> ev_panel, ev_wide;
  std::vector<int64_t> step_k, step_w;   // blocked schedule
  int* pairs = nullptr;                  // per-step net row movement
  bool lookahead = false;                // GELIM_LOOKAHEAD=1: side-stream wide updates
  bool fused = true;                     // GELIM_SCHEDULE=classic: separate update kernels
  bool narrow = true;                    // next panel's strip updated by the narrow kernel
  bool resident = false;                 // resident LU (rlu.hip): the default for n <= 1024
  int64_t split = 0;                     // hybrid: fused steps for columns < split, then the
                                         // resident LU on the trailing (n - split) system
  void* rws = nullptr;                   // its hand-off workspace
  double* sbuf = nullptr;                // narrow-update strip buffers (2 x 16 x ldL, column-major, ping-pong)
  double* lbuf = nullptr;                // fused steps: factored panels, column-major, ping-pong
  int64_t ldL = 0;                       //   (2 x 16 x ldL doubles)
  // wide-panel engine (n > big_tail): columns [0, big_k) are eliminated by
  // 256-column outer panels of 32-column multi-workgroup leaves (biglu.hip)
  // with fp64 MFMA trailing updates (dgemm.hip); the trailing
  // (n - big_k)-order system is solved by a nested plan of this file and the
  // top rows by one mat-vec + back substitution.
  int64_t big_k = 0;
  gelim_gauss_plan* tail = nullptr;
  void* big_ws = nullptr;                // leaf exchange granules + rows
  int* big_pairs = nullptr;              // per-leaf row movement
  double* big_y = nullptr;               // top right-hand side after the tail
  // lookahead (default from n = 3072, GELIM_BIG_LOOKAHEAD=0/1 forces it;
  // otherwise serial, graph-captured): the
  // trailing updates run on big_side, eagerly launched, every side kernel on
  // a grid of at most big_cap workgroups of one per CU (the CU count less
  // GELIM_BIG_RESERVE, default 64), so the leaf chain always finds free CUs
  bool big_la = false;
  int big_cap = 0;
  int* big_net = nullptr;                // an outer panel's composed row movement (side stream)
  hipStream_t big_side = nullptr;
  std::vector<hipEvent_t> big_ev;        // fork, fact[T], next[T], join
  hipGraphExec_t exec = nullptr;
  // the graph is captured ONCE on plan-owned buffers: the input is staged
  // into work and x / bnorm leave through xbuf / bnbuf, by eager copies
  // outside it (capturing the caller's pointers and re-capturing whenever
  // they changed corrupted results with two plans alive on ROCm 7.2,
  // profiles/graph_recapture.txt)
  double* xbuf = nullptr;
  double* bnbuf = nullptr;
  hipGraphExec_t exec_bn[2] = {nullptr, nullptr};  // fixed-pointer graphs without / with bnorm
};

namespace {

void retire_exec(hipGraphExec_t e) {
  if (e) (void)hipGraphExecDestroy(e);
}

constexpr int64_t kPairSlot = 72;  // 1 + 4*16 ints, padded

// Hybrid hand-off: perm[i] = i for the fused part (rows already in LAPACK
// order), split + piv[i] for the resident part (its pivot rows are physical
// rows of the trailing block); the resident kernel's singular column and
// hand-off error (info[2], info[3]) are folded into info[0], info[1].
//
// The resident part's row map is valid only when its kernel ran to the end
// (info[3] == 0): after an aborted hand-off the entries are whatever the last
// solve left (already offset by split), so they are replaced by the
// identity and info[1] keeps the abort code; an entry outside the trailing
// block is flagged as code 6.  Either way the back substitution never
// follows a row index outside the system.
__global__ void hybrid_perm_kernel(int* __restrict__ perm, int n, int split, int* __restrict__ info) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool aborted = info[3] != 0;
  if (i < n) {
    int v = i;
    if (i >= split && !aborted) {
      const int loc = perm[i];
      if (loc >= 0 && loc < n - split) v = split + loc;
      else atomicCAS(info + 1, 0, 6);
    }
    perm[i] = v;
  }
  if (i == 0) {
    if (info[0] == 0 && info[2] != 0) info[0] = split + info[2];
    if (info[1] == 0 && info[3] != 0) info[1] = info[3];
  }
}

// outer panel width of the wide-panel engine: 128 under the lookahead
// schedule up to n = 10240, 256 above it and under the serial schedule, 1024
// from n = 24576 on.  Measured with lookahead (profiles/big_nb_lookahead.txt):
// 8192 128 / 256 / 512 -> 34.2 / 34.8 / 41.1 ms; memplus (n = 17758) 169 /
// 151 ms for 128 / 256; serial 8192: 43.1 / 41.9 / 42.2 ms; round 5, 256 /
// 512 / 1024: 20480 219.3 / 227.4 / 229.6 ms, 24576 362.5 / 356.5 / 356.1 ms,
// 32768 845.0 / 797.5 / 785.8 ms (the K = nb trailing updates read and write
// all of C once per outer panel: 17 GB per update at 32768).
int64_t big_nb(bool la, int64_t n) {
  if (n >= 24576) return 1024;
  return (la && n <= 10240) ? int64_t(128) : int64_t(256);
}
constexpr int64_t kBigPairSlot = 1 + 4 * 32 + 3;

int enqueue(gelim_gauss_plan* p, const void* src, int64_t src_ld, void* dx, void* bnorm, hipStream_t s);

// U12 of outer panel [k, kend) on columns [cb, ce) (blocked forward
// substitution with the panel's unit-lower L11, one leaf-row block at a
// time), then their trailing update A[kend:, cb:ce) -= L21 U12 (K = kend - k).
int panel_u12_update(gelim_gauss_plan* p, double* A, int64_t k, int64_t kend, int64_t cb, int64_t ce,
                     hipStream_t s, int cap = 0) {
  using namespace gelim;
  const int64_t n = p->n, lda = p->lda, LW = big::leaf_width();
  if (ce <= cb) return GELIM_OK;
  if (big::trsm_fused() && kend - k <= 256) {  // the one-launch TRSM holds <= 256 rows in LDS
    GELIM_TRY(big::panel_trsm(A + k * lda + cb, lda, ce - cb, kend - k, A + k * lda + k, lda, s, cap));
  } else {
    for (int64_t r = k; r < kend; r += LW) {
      GELIM_TRY(big::laswp_trsm(A + r * lda, lda, r, 0, 0, cb, ce, ce, n - r, nullptr, s));
      if (r + LW < kend)
        GELIM_TRY(dgemm(A + (r + LW) * lda + cb, lda, A + (r + LW) * lda + r, lda, A + r * lda + cb, lda,
                        kend - r - LW, ce - cb, LW, -1.0, s));
    }
  }
  return dgemm_capped(A + kend * lda + cb, lda, A + kend * lda + k, lda, A + k * lda + cb, lda, n - kend, ce - cb,
                      kend - k, -1.0, cap, s);
}

// Wide-panel LU of columns [0, big_k) of the working system, then the tail
// solve and the block back substitution:
//   x[K..n) = tail solve of A[K:, K:] (already carrying every update),
//   y = A[0:K, n] - A[0:K, K:n] x[K..n),  x[0..K) = U11^-1 y.
//
// Outer panels P_j = [k_j, k_j+1) of big_nb(la, n) columns, each factored as
// 32-column leaves: per leaf the leaf itself (biglu.hip), its row movement
// on the other columns + the TRSM of its U rows, and a rank-32 GEMM of the
// columns right of it inside the panel.
//
// Serial schedule (n < 3072, or GELIM_BIG_LOOKAHEAD=0): after P_j, U12 and one K = 256
// GEMM update every column right of it -- the leaf chain and the big GEMMs
// alternate on one stream.
//
// Lookahead schedule (n >= 3072, or GELIM_BIG_LOOKAHEAD=1), the leaf chain on the caller's stream
// ("crit"), the big GEMMs beside it on big_side:
//   crit, P_j:  every leaf also updates the NEXT panel's columns P_j+1
//               (swap, TRSM, rank-32 GEMM -- right-looking at nb = 32), so
//               P_j+1 is ready the moment P_j's last leaf is; before its
//               first touch of P_j+1 it waits for side j-1's first part.
//   side, P_j:  after P_j's leaves, first P_j+2's columns (swaps, U12, K = 256
//               GEMM; event next[j]), then the L part left of P_j (swaps
//               only) and every column from P_j+3 on (swaps, U12, GEMM).
// Column sets never overlap between the streams while both run: crit owns
// P_j and P_j+1, side P_j+2 (until next[j]) and everything else.
int enqueue_big(gelim_gauss_plan* p, double* A, double* x, double* bnorm, hipStream_t s) {
  using namespace gelim;
  const int64_t n = p->n, lda = p->lda, K = p->big_k, LW = big::leaf_width();
  const int64_t nbw = big_nb(p->big_la, n);
  const int64_t T = (K + nbw - 1) / nbw;
  auto kb = [&](int64_t j) { return std::min(j * nbw, K); };  // P_j = [kb(j), kb(j+1))
  const bool la = p->big_la;
  hipStream_t side = la ? p->big_side : s;
  hipEvent_t* ev_fork = la ? &p->big_ev[0] : nullptr;
  hipEvent_t* ev_fact = la ? &p->big_ev[1] : nullptr;
  hipEvent_t* ev_next = la ? &p->big_ev[1 + T] : nullptr;
  hipEvent_t* ev_join = la ? &p->big_ev[1 + 2 * T] : nullptr;
  GELIM_TRY(zero_async(p->big_ws, big::workspace_bytes(), s));
  if (la) {
    HIP_TRY(hipEventRecord(*ev_fork, s));
    HIP_TRY(hipStreamWaitEvent(side, *ev_fork, 0));
  }
  int leaf = 0;
  for (int64_t j = 0; j < T; ++j) {
    const int64_t k = kb(j), kend = kb(j + 1);
    const int64_t cend = la ? kb(j + 2) : n + 1;  // columns the leaves update: P_j (+ P_j+1)
    const int first_leaf = leaf;
    for (int64_t c0 = k; c0 < kend; c0 += LW, ++leaf) {
      int* pr = p->big_pairs + leaf * kBigPairSlot;
      GELIM_TRY(big::leaf_factor(A + c0 * lda + c0, lda, n - c0, c0, p->pivot, p->piv, pr, p->info, p->big_ws,
                                 leaf, s));
      // P_j+1 is side j-1's until next[j-1]
      if (la && c0 == k && j > 0 && cend > kend) HIP_TRY(hipStreamWaitEvent(s, ev_next[j - 1], 0));
      // serial: interchanges on every other column (L part, rest of the
      // panel, trailing columns, b), TRSM inside the panel; lookahead: the
      // panel's own L part and P_j, P_j+1 (swaps + TRSM)
      GELIM_TRY(big::laswp_trsm(A + c0 * lda, lda, c0, la ? k : 0, c0, c0 + LW, cend, la ? cend : kend, n - c0, pr,
                                s));
      const int64_t c1 = c0 + LW;
      const int64_t gend = la ? cend : kend;
      if (c1 < gend)
        GELIM_TRY(dgemm(A + c1 * lda + c1, lda, A + c1 * lda + c0, lda, A + c0 * lda + c1, lda, n - c1, gend - c1, LW,
                        -1.0, s));
    }
    if (!la) {
      // U12 of the outer panel (its rows are final only now) and the
      // trailing update of every column right of it, b included
      GELIM_TRY(panel_u12_update(p, A, k, kend, kend, n + 1, s));
      continue;
    }
    const int nl = leaf - first_leaf;
    const int* pr0 = p->big_pairs + first_leaf * kBigPairSlot;
    HIP_TRY(hipEventRecord(ev_fact[j], s));
    HIP_TRY(hipStreamWaitEvent(side, ev_fact[j], 0));
    // the panel's row movement composed into one permutation (<= 64 rows per
    // leaf), applied by gather/scatter tiles; laswp_panel replays the lists
    const bool net = p->big_net != nullptr && nl * 2 * LW <= big::laswp_net_max() && n - k <= big::compose_max_rows();
    if (net) GELIM_TRY(big::compose_pairs(n, k, nl, pr0, kBigPairSlot, p->big_net, side));
    auto swaps = [&](int64_t lb, int64_t le, int64_t rb, int64_t re) {
      return net ? big::laswp_net(A + k * lda, lda, p->big_net, lb, le, rb, re, side, p->big_cap)
                 : big::laswp_panel(A, lda, n, k, nl, pr0, kBigPairSlot, lb, le, rb, re, side, p->big_cap);
    };
    // side, first part: P_j+2 = [kb(j+2), kb(j+3))
    const int64_t nb0 = kb(j + 2), nb1 = kb(j + 3);
    if (nb1 > nb0) {
      GELIM_TRY(swaps(0, 0, nb0, nb1));
      GELIM_TRY(panel_u12_update(p, A, k, kend, nb0, nb1, side, p->big_cap));
    }
    HIP_TRY(hipEventRecord(ev_next[j], side));
    // side, the rest: the L part left of P_j, every column from P_j+3 on
    const int64_t rb = std::max(nb1, cend);
    GELIM_TRY(swaps(0, k, rb, n + 1));
    GELIM_TRY(panel_u12_update(p, A, k, kend, rb, n + 1, side, p->big_cap));
  }
  if (la) {
    HIP_TRY(hipEventRecord(*ev_join, side));
    HIP_TRY(hipStreamWaitEvent(s, *ev_join, 0));
  }
  GELIM_TRY(enqueue(p->tail, A + K * lda + K, lda, x + K, bnorm ? bnorm + K : nullptr, s));
  GELIM_TRY(big::fold_info(p->info, p->tail->info, K, s));
  GELIM_TRY(big::tail_gemv(A, lda, n, K, x, p->big_y, bnorm, s));
  return backsub_f64(A, lda, p->big_y, 1, x, nullptr, K, 0, p->yw, s, nullptr, p->info + 1);
}

int enqueue(gelim_gauss_plan* p, const void* src, int64_t src_ld, void* dx, void* bnorm,
            hipStream_t s) {
  using namespace gelim;
  const int64_t n = p->n, lda = p->lda;
  if (p->big_k > 0) {
    if (src)
      GELIM_TRY(copy2d_async(p->work, lda * 8, src, src_ld * 8, (n + 1) * 8, n, s));
    GELIM_TRY(zero_async(p->info, 16, s));
    return enqueue_big(p, static_cast<double*>(p->work), static_cast<double*>(dx), static_cast<double*>(bnorm), s);
  }
  if (p->algo == GELIM_GPU_BLOCKED && p->resident) {
    // One persistent launch reads the system straight from src (no copy),
    // leaves U rows at their physical positions and the pivot row of every
    // column in piv; the persistent back substitution follows through piv.
    double* A = static_cast<double*>(p->work);
    GELIM_TRY(zero_async(p->info, 16, s));
    GELIM_TRY(rlu_factor(static_cast<const double*>(src), src_ld, A, lda, n, p->pivot, p->piv, p->info,
                         p->rws, s));
    return backsub_f64(A, lda, A + n, lda, static_cast<double*>(dx), static_cast<double*>(bnorm), n, 0,
                       p->yw, s, p->piv, p->info + 1);
  }
  if (src)
    GELIM_TRY(copy2d_async(p->work, lda * p->eb, src, src_ld * p->eb, (n + 1) * p->eb, n, s));
  const bool fused_hyb = p->algo == GELIM_GPU_BLOCKED && p->fused && p->split > 0 && p->split < n;
  if (fused_hyb) {
    // one prologue launch: the status words, the resident LU's flags and the
    // back substitution's sentinel-filled x (each its own launch otherwise)
    const unsigned sw = backsub_sentinel_word();
    const WordFill f[3] = {{p->info, 16, 0u}, rlu_flags_fill(n - p->split, p->rws), {dx, sizeof(double) * n, sw}};
    GELIM_TRY(fill_words_async(f, 3, s));
  } else {
    GELIM_TRY(zero_async(p->info, 16, s));
  }
  if (p->algo == GELIM_GPU_BLOCKED && p->fused) {
    // One fused launch per step (lu_step): workgroup 0 finishes step i-1 on
    // panel i's columns and factors panel i while the other workgroups apply
    // step i-1 to the columns right of panel i; a closing launch applies the
    // last step to b.  S+1 launches, stream-ordered, no events.
    // With narrow (default) a small many-workgroup kernel between the steps
    // applies step i to panel i+1's strip, so the panel workgroup starts on
    // an up-to-date strip.
    double* A = static_cast<double*>(p->work);
    const bool hyb = p->split > 0 && p->split < n;
    // hybrid: only the steps left of the split run here; the closing launch
    // applies the last of them to every column from the split on (b too)
    size_t S = p->step_k.size();
    if (hyb) S = (size_t)(std::lower_bound(p->step_k.begin(), p->step_k.end(), p->split) - p->step_k.begin());
    const int64_t kend = hyb ? p->split : n;
    const bool nar = p->narrow;
    // step i writes its factored panel to lbuf[i % 2]; step i + 1's trailing
    // updates and narrow(i) read it there
    auto lb = [&](size_t i) { return p->lbuf + (i & 1) * 16 * p->ldL; };
    // narrow(i)'s output: read by step i + 1's panel workgroup while the fused
    // narrow(i + 1) of that same launch writes the other buffer
    auto sb = [&](size_t i) { return p->sbuf + (i & 1) * 16 * p->ldL; };
    // (the narrow update fused into the step launch through flag hand-offs
    // measured equal, 3.77 vs 3.76 ms, profiles/headline_2048_r4.md)
    for (size_t i = 0; i <= S; ++i) {
      const int64_t kp = i ? p->step_k[i - 1] : 0, wp = i ? p->step_w[i - 1] : 0;
      const int64_t k = i < S ? p->step_k[i] : kend, w = i < S ? p->step_w[i] : 0;
      const int* prev = i ? p->pairs + (i - 1) * kPairSlot : nullptr;
      int* cur = i < S ? p->pairs + i * kPairSlot : nullptr;
      const bool nx = nar && i + 1 < S;  // a narrow update of panel i + 1's strip follows step i
      GELIM_TRY(lu_step(A, lda, n, kp, wp, prev, k, w, p->pivot, p->piv, p->info, cur, s,
                        nar && i ? sb(i - 1) : nullptr, i < S ? lb(i) : nullptr, i ? lb(i - 1) : nullptr,
                        p->ldL, nullptr, sb(i), nx ? p->step_k[i + 1] : 0,
                        nx ? p->step_w[i + 1] : 0));
      if (nx)
        GELIM_TRY(lu_narrow(A, lda, n, k, w, cur, p->step_k[i + 1], p->step_w[i + 1], sb(i), s,
                            lb(i), p->ldL));
    }
    if (hyb) {
      // the trailing (n - split) system, fully updated, factored in place by
      // the resident LU (one persistent launch; faster than the step
      // launches once the panel fits 2 register slots); one back
      // substitution over both parts through the merged row map
      const int64_t K = p->split;
      GELIM_TRY(rlu_factor(nullptr, 0, A + K * lda + K, lda, n - K, p->pivot, p->piv + K, p->info + 2,
                           p->rws, s, nullptr, /*flags_ready=*/true));
      hipLaunchKernelGGL(hybrid_perm_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p->piv,
                         (int)n, (int)K, p->info);
      HIP_TRY(hipGetLastError());
      return backsub_f64(A, lda, A + n, lda, static_cast<double*>(dx), static_cast<double*>(bnorm), n, 0,
                         p->yw, s, p->piv, p->info + 1, /*x_ready=*/true);
    }
    return backsub_f64(A, lda, A + n, lda, static_cast<double*>(dx),
                       static_cast<double*>(bnorm), n, 0, p->yw, s);
  }
  if (p->algo == GELIM_GPU_BLOCKED) {
    // Right-looking blocked LU with lookahead 1.  Critical stream s:
    //   panel(i) -> [wait wide(i-1)] -> narrow(i) -> panel(i+1) -> ...
    // where narrow(i) applies panel i to the NEXT panel's columns only;
    // side stream: [wait panel(i)] -> wide(i) = panel i applied to every
    // column right of the next panel (incl. b).  The wide GEMM of step i
    // runs under the single-CU panel factorisation of step i+1.
    double* A = static_cast<double*>(p->work);
    const size_t S = p->step_k.size();
    const bool la = p->lookahead;
    hipStream_t side = la ? p->side : s;
    if (la) {
      HIP_TRY(hipEventRecord(p->ev_wide[S], s));  // fork: side joins the stream/capture
      HIP_TRY(hipStreamWaitEvent(side, p->ev_wide[S], 0));
    }
    for (size_t i = 0; i < S; ++i) {
      const int64_t k = p->step_k[i], w = p->step_w[i], m = n - k;
      int* pr = p->pairs + i * kPairSlot;
      GELIM_TRY(panel_factor(A + k * lda + k, lda, m, w, k, p->pivot, p->piv + k, p->info, s, pr));
      if (la) HIP_TRY(hipEventRecord(p->ev_panel[i], s));
      const int64_t kn = k + w;                                      // next panel's first column
      const int64_t wn = (la && i + 1 < S) ? p->step_w[i + 1] : 0;  // narrow width (lookahead only)
      // side: wide update of columns [kn + wn, n] (b included)
      if (la) HIP_TRY(hipStreamWaitEvent(side, p->ev_panel[i], 0));
      const int64_t wc0 = kn + wn, wcols = (n + 1) - wc0;
      if (wcols > 0) {
        GELIM_TRY(pairs_trsm(A + k * lda + wc0, lda, wcols, A + k * lda + k, lda, w, pr, side));
        if (m > w)
          GELIM_TRY(gemm_update(A + kn * lda + wc0, lda, A + kn * lda + k, lda, A + k * lda + wc0,
                                lda, m - w, wcols, w, side));
      }
      if (la) HIP_TRY(hipEventRecord(p->ev_wide[i], side));
      // critical: narrow update of the next panel's columns [kn, kn + wn)
      if (wn > 0) {
        if (la && i > 0) HIP_TRY(hipStreamWaitEvent(s, p->ev_wide[i - 1], 0));
        GELIM_TRY(pairs_trsm(A + k * lda + kn, lda, wn, A + k * lda + k, lda, w, pr, s));
        GELIM_TRY(gemm_update(A + kn * lda + kn, lda, A + kn * lda + k, lda, A + k * lda + kn, lda,
                              m - w, wn, w, s));
      }
    }
    if (la) HIP_TRY(hipStreamWaitEvent(s, p->ev_wide[S - 1], 0));  // join
    return backsub_f64(A, lda, A + n, lda, static_cast<double*>(dx),
                       static_cast<double*>(bnorm), n, 0, p->yw, s);
  }
  // hip-pivot: one persistent launch for the whole elimination when the
  // system fits the chip's registers (n <= 2048) and the grid is
  // co-resident (pivot_persist.hip), else two launches per column
  if (p->eb == 8) {
    double* A = static_cast<double*>(p->work);
    int rc = pivot_persistent<double>(A, lda, n, p->pivot, p->info, p->piv, p->diag, p->pws, s);
    if (rc < 0) return rc;
    if (rc == 1)
      GELIM_TRY(pivot_elimination<double>(A, lda, n, p->pivot, static_cast<double*>(p->mcol),
                                          p->info, s, p->piv, p->diag));
    return backsub_f64(A, lda, A + n, lda, static_cast<double*>(dx),
                       static_cast<double*>(bnorm), n, 1, p->yw, s);
  }
  float* A = static_cast<float*>(p->work);
  int rc = pivot_persistent<float>(A, lda, n, p->pivot, p->info, p->piv, p->diag, p->pws, s);
  if (rc < 0) return rc;
  if (rc == 1)
    GELIM_TRY(pivot_elimination<float>(A, lda, n, p->pivot, static_cast<float*>(p->mcol), p->info,
                                       s, p->piv, p->diag));
  return backsub_f32(A, lda, A + n, lda, static_cast<double*>(dx), static_cast<double*>(bnorm), n,
                     1, p->yw, s);
}

}  // namespace

extern "C" gelim_gauss_plan* gelim_gauss_plan_create(int64_t n, int algo, int pivot,
                                                     int dtype_bytes, int use_graph) {
  if (n <= 0 || (dtype_bytes != 4 && dtype_bytes != 8) ||
      (algo != GELIM_GPU_BLOCKED && algo != GELIM_GPU_PIVOT) ||
      (pivot != GELIM_PIVOT_ZERO && pivot != GELIM_PIVOT_PARTIAL)) {
    GELIM_FAIL(GELIM_E_ARG, "plan_create: bad arguments");
    return nullptr;
  }
  if (algo == GELIM_GPU_BLOCKED && dtype_bytes != 8) {
    GELIM_FAIL(GELIM_E_ARG, "blocked LU is fp64 only (fp32 fails saylr4/orsreg_1, SURVEY §4.3)");
    return nullptr;
  }
  // wide-panel engine for n > big_tail (default 2048, the largest order the
  // register-resident engines take; GELIM_BIG_TAIL lowers it for tests):
  // columns [0, big_k) with big_k the multiple of the leaf width that leaves
  // a trailing system of at most big_tail
  int64_t big_tail = 2048;
  if (const char* e = std::getenv("GELIM_BIG_TAIL")) big_tail = std::max<int64_t>(64, std::min<int64_t>(2048, std::atoll(e)));
  const int64_t lw = gelim::big::leaf_width();
  const int64_t big_k = (algo == GELIM_GPU_BLOCKED && n > big_tail) ? (n - big_tail + lw - 1) / lw * lw : 0;
  if (big_k > 0 && n > gelim::big::max_rows()) {
    GELIM_FAIL(GELIM_E_ARG, "blocked LU: n > " + std::to_string(gelim::big::max_rows()) + " not supported on one GPU");
    return nullptr;
  }
  auto* p = new gelim_gauss_plan;
  p->n = n;
  p->algo = algo;
  p->pivot = pivot;
  p->eb = dtype_bytes;
  p->use_graph = use_graph != 0;
  const int64_t align = 64 / dtype_bytes;  // 64-byte rows
  // the wide-panel engine's GEMMs read 16-byte chunks that may reach one
  // column past b: keep at least one padding column
  p->lda = (n + 1 + (big_k > 0 ? 1 : 0) + align - 1) / align * align;
  auto fail = [&](const char* what) -> gelim_gauss_plan* {
    GELIM_FAIL(GELIM_E_NOMEM, std::string("plan_create: ") + what);
    gelim_gauss_plan_destroy(p);
    return nullptr;
  };
  if (big_k > 0) {
    p->big_k = big_k;
    if (hipMalloc(&p->work, (size_t)(n * p->lda * 8)) != hipSuccess) return fail("work");
    if (hipMalloc((void**)&p->piv, (size_t)(n + 64) * sizeof(int)) != hipSuccess) return fail("piv");
    if (hipMalloc((void**)&p->info, 16) != hipSuccess) return fail("info");
    if (hipMalloc((void**)&p->yw, (size_t)n * sizeof(double)) != hipSuccess) return fail("yw");
    if (hipMalloc((void**)&p->big_y, (size_t)big_k * sizeof(double)) != hipSuccess) return fail("big_y");
    if (hipMalloc(&p->big_ws, gelim::big::workspace_bytes()) != hipSuccess) return fail("leaf workspace");
    const int64_t nleaves = big_k / lw;
    if (hipMalloc((void**)&p->big_pairs, sizeof(int) * kBigPairSlot * nleaves) != hipSuccess) return fail("pairs");
    if (hipStreamCreateWithFlags(&p->cap, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    // lookahead: trailing updates on a second stream, launched eagerly.  Every side kernel runs on a capped grid of one workgroup per
    // CU (dgemm_capped, panel_trsm, laswp_panel with max_wg), so at most
    // big_cap CUs ever hold side work and the leaf chain -- whose waves need
    // a whole SIMD's registers and all of a leaf's workgroups resident --
    // always finds free CUs.  Earlier attempts (profiles/big_lookahead_8192.txt):
    // uncapped grids 42.3 ms (leaves dispatched only as GEMM workgroups
    // drained), a CU-masked side queue 147 ms (it never ran beside the leaves).
    // default: lookahead from n = 3072 (with the 128-column outer panels,
    // profiles/big_nb_lookahead.txt: 3072 8.45 vs 8.57 ms serial, 4096 12.9
    // vs 13.5, 5120 17.7 vs 19.1, 8192 34.2 vs 39.9)
    const char* el = std::getenv("GELIM_BIG_LOOKAHEAD");
    p->big_la = el ? std::atoi(el) != 0 : n >= 3072;
    if (p->big_la) {
      int dev = 0, ncu = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      int reserve = 64;  // 8192: 35.4 ms (32: 36.3, 96: 35.5)
      // never fewer free CUs than the first (largest) leaf needs at once: a
      // side GEMM holds its CUs for its whole grid-stride loop, and a leaf
      // whose participants cannot all be resident would spin into its timeout
      reserve = std::max(reserve, gelim::big::leaf_cus(n) + 8);
      p->big_cap = ncu > reserve + 8 ? ncu - reserve : std::max(8, ncu / 2);
      if (gelim::side_stream_create(&p->big_side) != GELIM_OK) return fail("side stream");
      if (hipMalloc((void**)&p->big_net, sizeof(int) * (1 + 2 * (size_t)gelim::big::laswp_net_max())) != hipSuccess)
        return fail("net movement");
      const int64_t T = (big_k + big_nb(true, n) - 1) / big_nb(true, n);
      p->big_ev.assign((size_t)(2 * T + 2), nullptr);
      for (auto& e : p->big_ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail("event");
    }
    p->tail = gelim_gauss_plan_create(n - big_k, algo, pivot, dtype_bytes, 0);
    if (!p->tail) {
      gelim_gauss_plan_destroy(p);
      return nullptr;
    }
    (void)hipMemset(p->work, 0, (size_t)(n * p->lda * 8));
    return p;
  }
  if (hipMalloc(&p->work, (size_t)(n * p->lda * dtype_bytes)) != hipSuccess) return fail("work");
  if (hipMalloc((void**)&p->piv, (size_t)(n + 64) * sizeof(int)) != hipSuccess) return fail("piv");
  if (hipMalloc((void**)&p->info, 16) != hipSuccess) return fail("info");
  if (hipMalloc((void**)&p->yw, (size_t)n * sizeof(double)) != hipSuccess) return fail("yw");
  if (hipMalloc(&p->mcol, (size_t)n * dtype_bytes) != hipSuccess) return fail("mcol");
  if (hipMalloc((void**)&p->diag, (size_t)n * sizeof(double)) != hipSuccess) return fail("diag");
  if (hipMalloc(&p->ry, (size_t)n * dtype_bytes) != hipSuccess) return fail("ry");
  if (hipMalloc((void**)&p->tmp, (size_t)2 * 32 * (n + 1) * sizeof(double)) != hipSuccess)
    return fail("tmp");
  if (hipStreamCreateWithFlags(&p->cap, hipStreamNonBlocking) != hipSuccess) return fail("stream");
  if (algo == GELIM_GPU_PIVOT && hipMalloc(&p->pws, gelim::pivot_persist_ws_bytes(n)) != hipSuccess)
    return fail("pivot exchange buffers");
  if (const char* e = std::getenv("GELIM_LOOKAHEAD")) p->lookahead = std::atoi(e) != 0;
  if (const char* e = std::getenv("GELIM_SCHEDULE")) p->fused = std::string(e) != "classic";
  if (p->lookahead) p->fused = false;
  {
    // GELIM_SCHEDULE: auto (default) | resident | fused | classic.  auto =
    // the resident LU up to n = 1024 (R <= 2 register slots: measured 0.73
    // vs 0.93 ms at 512, 1.58 vs 2.06 ms at 1024) and the fused step
    // schedule above (at R = 4 the resident engine's strip update spills and
    // its scalar-cache broadcasts are latency-bound: 6.1 vs 4.95 ms at 2048,
    // profiles/rlu_phase_stamps.txt).  resident forces it up to 2048.
    const char* e = std::getenv("GELIM_SCHEDULE");
    const std::string sched = e ? e : "auto";
    const int64_t lim = sched == "resident" ? gelim::rlu_max_n() : sched == "auto" ? 1024 : 0;
    p->resident = algo == GELIM_GPU_BLOCKED && n <= lim && !p->lookahead && gelim::rlu_coresident(n);
    // GELIM_HYBRID: rows of the trailing system handed to the resident LU
    // (default 1024, its 2-slot regime; 0 = off, pure fused schedule; any
    // other value up to 2048, rounded to a panel boundary -- 1, 2 and 4
    // register slots, each covered by a GPU test)
    const char* eh = std::getenv("GELIM_HYBRID");
    const int64_t tail = eh ? std::max<int64_t>(0, std::min<int64_t>(gelim::rlu_max_n(), std::atoll(eh))) : 1024;
    if (algo == GELIM_GPU_BLOCKED && !p->resident && p->fused && tail > 0 && n > tail &&
        tail <= gelim::rlu_max_n() && sched != "fused" && gelim::rlu_coresident(tail))
      p->split = n - tail;  // rounded to a panel boundary below
  }
  if (algo == GELIM_GPU_BLOCKED) {
    for (int64_t k = 0; k < n;) {
      const int64_t w = std::min<int64_t>(gelim::panel_width_for(n - k), n - k);
      p->step_k.push_back(k);
      p->step_w.push_back(w);
      k += w;
    }
    if (p->split > 0) {  // first panel start with at most `tail` rows below it
      const int64_t want = p->split;
      p->split = n;
      for (int64_t k : p->step_k)
        if (k >= want) {
          p->split = k;
          break;
        }
    }
    const size_t S = p->step_k.size();
    if (gelim::side_stream_create(&p->side) != GELIM_OK) return fail("side");
    p->ev_panel.assign(S, nullptr);
    p->ev_wide.assign(S + 1, nullptr);
    for (auto* v : {&p->ev_panel, &p->ev_wide})
      for (auto& e : *v)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail("event");
    if (hipMalloc((void**)&p->pairs, sizeof(int) * kPairSlot * S) != hipSuccess) return fail("pairs");
    p->ldL = gelim::lu_panel_buffer_ld(n);
    if (hipMalloc((void**)&p->sbuf, sizeof(double) * 2 * 16 * p->ldL) != hipSuccess) return fail("sbuf");
    if (hipMalloc((void**)&p->lbuf, sizeof(double) * 2 * 16 * p->ldL) != hipSuccess) return fail("lbuf");
    if (p->resident && hipMalloc(&p->rws, gelim::rlu_workspace_bytes(n)) != hipSuccess)
      return fail("resident LU workspace");
    if (!p->resident && p->split > 0 && p->split < n &&
        hipMalloc(&p->rws, gelim::rlu_workspace_bytes(n - p->split)) != hipSuccess)
      return fail("resident LU workspace (hybrid)");
  }
  (void)hipMemset(p->work, 0, (size_t)(n * p->lda * dtype_bytes));
  return p;
}

extern "C" void gelim_gauss_plan_destroy(gelim_gauss_plan* p) {
  if (!p) return;
  retire_exec(p->exec);
  for (auto& e : p->exec_bn) retire_exec(e);
  (void)hipFree(p->xbuf);
  (void)hipFree(p->bnbuf);
  if (p->cap) (void)hipStreamDestroy(p->cap);
  if (p->side) (void)hipStreamDestroy(p->side);
  if (p->big_side) (void)hipStreamDestroy(p->big_side);
  for (auto& e : p->big_ev)
    if (e) (void)hipEventDestroy(e);
  for (auto* v : {&p->ev_panel, &p->ev_wide})
    for (auto& e : *v)
      if (e) (void)hipEventDestroy(e);
  (void)hipFree(p->pairs);
  (void)hipFree(p->sbuf);
  (void)hipFree(p->lbuf);
  (void)hipFree(p->rws);
  (void)hipFree(p->work);
  (void)hipFree(p->piv);
  (void)hipFree(p->info);
  (void)hipFree(p->yw);
  (void)hipFree(p->mcol);
  (void)hipFree(p->diag);
  (void)hipFree(p->ry);
  (void)hipFree(p->tmp);
  (void)hipFree(p->pws);
  (void)hipFree(p->big_ws);
  (void)hipFree(p->big_pairs);
  (void)hipFree(p->big_net);
  (void)hipFree(p->big_y);
  gelim_gauss_plan_destroy(p->tail);
  delete p;
}

extern "C" int64_t gelim_gauss_plan_lda(const gelim_gauss_plan* p) { return p ? p->lda : 0; }
extern "C" void* gelim_gauss_plan_work(gelim_gauss_plan* p) { return p ? p->work : nullptr; }

extern "C" int gelim_gauss_plan_solve(gelim_gauss_plan* p, const void* src, int64_t src_ld,
                                      void* dx, void* bnorm, void* stream) {
  if (!p || !dx) return GELIM_FAIL(GELIM_E_ARG, "plan_solve: null plan or x");
  if (src && src_ld < p->n + 1) return GELIM_FAIL(GELIM_E_ARG, "plan_solve: src_ld < n+1");
  hipStream_t s = (hipStream_t)stream;
  if (!p->use_graph || p->big_la) return enqueue(p, src, src_ld, dx, bnorm, s);
  auto capture = [&](const void* csrc, int64_t cld, void* cdx, void* cbn) -> int {
    retire_exec(p->exec);
    p->exec = nullptr;
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(p->cap, hipStreamCaptureModeThreadLocal));
    int rc = enqueue(p, csrc, cld, cdx, cbn, p->cap);
    hipError_t e = hipStreamEndCapture(p->cap, &g);
    if (rc != 0) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    HIP_TRY(e);
    e = hipGraphInstantiate(&p->exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_TRY(e);
    return GELIM_OK;
  };
  // one graph per plan (and per bnorm on/off), on plan-owned buffers only
  const int64_t n = p->n;
  if (!p->xbuf) {
    HIP_TRY(hipMalloc((void**)&p->xbuf, sizeof(double) * n));
    HIP_TRY(hipMalloc((void**)&p->bnbuf, sizeof(double) * n));
  }
  const bool want_bn = bnorm != nullptr;
  hipGraphExec_t& ex = p->exec_bn[want_bn ? 1 : 0];
  if (!ex) {  // captured once, destroyed only with the plan
    GELIM_TRY(capture(nullptr, 0, p->xbuf, want_bn ? p->bnbuf : nullptr));
    ex = p->exec;
    p->exec = nullptr;
  }
  if (src)
    GELIM_TRY(gelim::copy2d_async(p->work, p->lda * p->eb, src, src_ld * p->eb, (n + 1) * p->eb, n, s));
  HIP_TRY(hipGraphLaunch(ex, s));
  GELIM_TRY(gelim::copy2d_async(dx, 0, p->xbuf, 0, sizeof(double) * n, 1, s));
  if (want_bn) GELIM_TRY(gelim::copy2d_async(bnorm, 0, p->bnbuf, 0, sizeof(double) * n, 1, s));
  return GELIM_OK;
}

// Re-solve A x = c with the factors the last hip-pivot solve left in the
// plan (O(n^2): permutation + lower solve + unit upper back substitution);
// c and x are fp64 device vectors.  The refinement loop of
// GaussSolver.solve_refined uses it instead of re-factoring.
extern "C" int gelim_gauss_plan_resolve(gelim_gauss_plan* p, const double* c, double* x, void* stream) {
  using namespace gelim;
  if (!p || !c || !x) return GELIM_FAIL(GELIM_E_ARG, "plan_resolve: null argument");
  if (p->algo != GELIM_GPU_PIVOT) return GELIM_FAIL(GELIM_E_ARG, "plan_resolve: only the hip-pivot plan keeps its factors");
  hipStream_t s = (hipStream_t)stream;
  const int64_t n = p->n, lda = p->lda;
  if (p->eb == 8) {
    const double* A = static_cast<const double*>(p->work);
    GELIM_TRY(pivot_lower_resolve<double>(A, lda, n, p->piv, p->diag, c, static_cast<double*>(p->ry), s));
    return backsub_f64(A, lda, static_cast<const double*>(p->ry), 1, x, nullptr, n, 1, p->yw, s);
  }
  const float* A = static_cast<const float*>(p->work);
  GELIM_TRY(pivot_lower_resolve<float>(A, lda, n, p->piv, p->diag, c, static_cast<float*>(p->ry), s));
  return backsub_f32(A, lda, static_cast<const float*>(p->ry), 1, x, nullptr, n, 1, p->yw, s);
}

extern "C" int gelim_gauss_plan_info(gelim_gauss_plan* p, void* stream) {
  if (!p) return GELIM_FAIL(GELIM_E_ARG, "plan_info: null plan");
  int h[4] = {0, 0, 0, 0};
  HIP_TRY(hipMemcpyAsync(h, p->info, 16, hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  if (h[1] == 8) return GELIM_FAIL(GELIM_E_HIP, "resident LU: an updater read a pivot row outside the system (code 8)");
  if (h[1] == 6 || h[1] == 7)
    return GELIM_FAIL(GELIM_E_HIP, std::string("row map out of range (code ") + std::to_string(h[1]) +
                                       (h[1] == 6 ? "): resident LU pivot outside its block"
                                                  : "): back substitution row map outside the system"));
  if (h[1] != 0)
    return GELIM_FAIL(GELIM_E_HIP, "GPU hand-off timed out (code " + std::to_string(h[1]) +
                                       "): workgroups of a persistent kernel were not co-resident");
  return h[0];
}
