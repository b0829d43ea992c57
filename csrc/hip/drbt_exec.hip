// Native executor of DistributedRBT's lookahead factorisation
// (parallel/dist_rbt.py _factor_lookahead, which stays the reference
// implementation for the host-rendezvous transports): the same schedule,
// issued from C++ on the solver's probed streams with a pool of events and
// libgelim's own RCCL communicators.
//
// Why native: issued from Python the loop costs ~120 us of host time per
// 128-column block (more than the GPU chain of a block at 8 ranks), and as a
// hipGraph replay the runtime maps the graph's branches onto hardware queues
// itself -- the chain's small kernels then queue behind side-stream GEMMs on
// a shared queue and every cross-queue edge costs 12-17 us
// (profiles/dist_rbt_replay_r6.md).  Issued here, each block is ~12 runtime
// calls (~30 us of host time, under the GPU chain) and every stream keeps
// the hardware queue it was probed onto.
//
// Per block k (owner o = k % P), column k goes out as three messages:
//   small_k = [Dinv_k; L_{k+1,k}]: on the MAIN stream through its own
//          communicator -- the chain is small_k -> W = Dinv_k M[k, k+1] ->
//          M[k+1,k+1] -= L_{k+1,k} W -> Dinv_{k+1} -> small_{k+1}, with no
//          cross-stream hop but the next-row product's (below);
//   next_k = L_{k+2,k} and rest_k = L_{k+3..,k}: on the COMM stream through a
//          second communicator.  The owner of k+1 computes the rows they
//          carry there too, beside its inverse: the next block row
//          M[k+2,k+1] -= L_{k+2,k} W (from next_k; small_{k+1} waits for it),
//          then M[k+3,k+1] (from rest_k's first block) -> next_{k+1}, then the
//          rest -> rest_{k+1}.  So the chain never waits on the bulk of a
//          column: rest_k has the two block steps before small_{k+2} to land.
// Every rank, side: [small_k, next_k, rest_k] panel k -> its next block
//   (ev_first), then the rest of its columns (ev_rest).
// Every product has dgemm.hip's per-element operation order (the 128-wide
// ones run as dgemm.hip tile16_kernel, bit-identical) and the inverses are the same
// kernel, so this schedule and the Python one (two messages per column) give
// the same factor bits (tests/test_gpu_dist_rbt.py::
// test_native_executor_matches_python, test_chain_products_match_dgemm).
//
// Replay (scripts/one_rank_of_p.py): rank r of a virtual P-rank run on one
// GPU -- every other rank's chain step runs here on a rotating scratch slab
// and every message is a device copy of the same size, so one GPU measures
// the chain plus the contention with rank r's side share.
//
// Reference: OpenMP_and_MPI/gauss_mpi/gauss_internal_input.c:141-175 (every
// worker updates rows at every pivot step; here every rank updates its own
// resident columns at every block step).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
int dgemm_launch(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
                 int64_t N, int64_t K, double alpha, int max_wg, hipStream_t s, int accumulate, int group_arg,
                 int64_t bbs, int64_t cbs);
}  // namespace gelim

extern "C" int gelim_rbt_block_inverse(const double* Ablk, int64_t lda, int64_t col, double* Dinv, int* info,
                                       void* stream);
extern "C" int gelim_rccl_bcast(void* comm, void* buf, int64_t count, int32_t dtype, int32_t root, void* stream);

// Mirrors parallel/dist_rbt.py (ctypes.Structure _ExecArgs); keep in sync.
struct gelim_drbt_args {
  int64_t np, nloc;
  int32_t P, rank;
  double* Mb;           // nloc / 128 slabs of np x 128, mbs doubles apart
  int64_t mbs;
  double* X[3];         // landing buffers, np x 128 each
  double* Wm;           // 2 x 128 x 128: the chain steps' W, a ring of two
  double* Ws;           // 128 x nloc (side)
  int32_t* info;        // device: 1 + first column of a non-finite inverse (atomicMin)
  void* main;           // hipStream_t (null: the default stream)
  void* side;
  void* comm;
  void* rccl_small;     // communicators (null: no collective -- one rank, or the replay)
  void* rccl_bulk;
  int32_t side_cap;     // CUs for the bulk GEMMs beside the chain: side, and the rows below on comm (0 = all)
  int32_t replay;       // 1: replay mode (module comment)
  double* F[3];         // replay: scratch slabs np x 128
  void* aux;            // replay: the virtual owners' side stream
  double* Wfs;          // replay: 2 x 128 x 128, the virtual owners' side W (a ring of two)
  int32_t* finfo;       // replay: the scratch inverses' info word
};

namespace {

// The chain's 128-wide products: C (M x 128, ldc) = A B (accumulate 0) or
// C -= A B (accumulate 1), K = 128, as dgemm.hip's 16 x 16 tiles (one
// 64-thread workgroup each, no LDS; bit-identical to dgemm): 64 workgroups
// for M = 128, 3.9 us against 8.6 for dgemm's 64-tile grid
// (profiles/dist_rbt_replay_r6.md).
int tile_gemm(double* C, int64_t ldc, const double* A, int64_t lda, const double* B, int64_t ldb, int64_t M,
              int accumulate, hipStream_t s) {
  return gelim::dgemm_tiles(gelim::GemmOp{C, ldc, A, lda, B, ldb, M, 128, 128}, gelim::GemmOp{}, accumulate ? -1.0 : 1.0,
                            accumulate, s);
}

}  // namespace

struct gelim_drbt_exec {
  int nb = 0;
  std::vector<hipEvent_t> ev;  // kNev per block
};

namespace {

constexpr int NB = 128;
// per block k: kSmall (main: small_k in place), kBulk (comm: next_k and rest_k
// in place, and the comm stream's reads of column k-1 done), kW (main: step
// k's W and diagonal update, or its receive), kNR (comm: block k+1's next
// block row), kFirst / kRest (side: panel k applied to the next local block /
// to every local block), kAuxSide (replay: the virtual owner of block k has
// applied panel k-2), kShipDone (replay: rest_k copied out of its scratch slab)
// kTop / kAuxTop: the same applies' first two block rows below k (all that
// the next chain step's main-stream products read).
// kNext: next_k in place (comm), all that the top rows' applies need besides small_k.
enum { kSmall, kNext, kBulk, kW, kNR, kTop, kFirst, kRest, kAuxTop, kAuxSide, kShipDone, kNev };

int mk_events(gelim_drbt_exec* ex, int nb) {
  if (ex->nb >= nb) return GELIM_OK;
  for (hipEvent_t e : ex->ev) (void)hipEventDestroy(e);
  ex->ev.assign((size_t)nb * kNev, nullptr);
  for (auto& e : ex->ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  ex->nb = nb;
  return GELIM_OK;
}

struct Exec {
  const gelim_drbt_args& a;
  gelim_drbt_exec* ex;
  hipStream_t main, side, comm, aux;
  int64_t nb, nbl;

  hipEvent_t ev(int64_t k, int which) const { return ex->ev[(size_t)k * kNev + which]; }
  bool owns(int64_t k) const { return k % a.P == a.rank; }
  double* col(int64_t k) const {  // column k from its diagonal block down (ld 128)
    return owns(k) ? a.Mb + (k / a.P) * a.mbs + k * NB * NB : a.X[k % 3];
  }
  double* wbuf(int64_t k) const { return a.Wm + (k & 1) * NB * NB; }  // step k's W (a ring of two)
  int64_t first_lb_after(int64_t k) const {
    const int64_t q = (k + 1 - a.rank + a.P - 1) / a.P;  // ceil((k + 1 - rank) / P), >= 0 here
    return std::min(nbl, std::max<int64_t>(0, k + 1 - a.rank > 0 ? q : 0));
  }

  int gemm(double* C, int64_t ldc, int64_t cbs, const double* A, int64_t lda, const double* B, int64_t ldb,
           int64_t bbs, int64_t M, int64_t N, int64_t K, double alpha, int acc, int cap, hipStream_t s) const {
    if (M <= 0 || N <= 0) return GELIM_OK;
    return gelim::dgemm_launch(C, ldc, A, lda, B, ldb, M, N, K, alpha, cap, s, acc, -1, bbs, cbs);
  }
  // W[:, :128 (lb1 - lb0)] = Dinv_k M[k, local blocks lb0 .. lb1)
  int panel_w(int64_t k, const double* c, int64_t lb0, int64_t lb1, double* W, int64_t ldw, hipStream_t s) const {
    return gemm(W, ldw, 0, c, NB, a.Mb + lb0 * a.mbs + k * NB * NB, NB, a.mbs, NB, (lb1 - lb0) * NB, NB, 1.0, 0, 0,
                s);
  }
  // M[r0:r1, local blocks lb0 .. lb1) -= L_k[r0:r1] W
  int panel_rows(int64_t k, const double* c, int64_t lb0, int64_t lb1, int64_t r0, int64_t r1, const double* W,
                 int64_t ldw, int cap, hipStream_t s) const {
    if (lb1 <= lb0 || r1 <= r0) return GELIM_OK;
    return gemm(a.Mb + lb0 * a.mbs + r0 * NB, NB, a.mbs, c + (r0 - k * NB) * NB, NB, W, ldw, 0, r1 - r0,
                (lb1 - lb0) * NB, NB, -1.0, 1, cap, s);
  }
  // panel k applied to local blocks lb0 .. lb1; with top, rows k+1 .. k+2
  // first, then the event top, then the rows below
  // (the caller has made s wait for small_k and next_k; the rows below
  // k+2 wait here for rest_k)
  int apply_panel(int64_t k, const double* c, int64_t lb0, int64_t lb1, double* W, int64_t ldw, int cap,
                  hipStream_t s, hipEvent_t top = nullptr) const {
    const int64_t r1 = top ? std::min(a.np, (k + 3) * NB) : (k + 1) * NB;
    if (lb1 > lb0) {
      GELIM_TRY(panel_w(k, c, lb0, lb1, W, ldw, s));
      GELIM_TRY(panel_rows(k, c, lb0, lb1, (k + 1) * NB, r1, W, ldw, cap, s));
    }
    if (top) HIP_TRY(hipEventRecord(top, s));
    HIP_TRY(hipStreamWaitEvent(s, ev(k, kBulk), 0));
    return lb1 > lb0 ? panel_rows(k, c, lb0, lb1, r1, a.np, W, ldw, cap, s) : GELIM_OK;
  }
  int invert(double* blk, int64_t colidx, int32_t* info, hipStream_t s) const {
    return gelim_rbt_block_inverse(blk, NB, colidx, blk, info, s);
  }

  // Row blocks [b0, b1) of column k to every rank, on stream s: the owner's
  // slab in place, receivers into their landing buffer (replay: a copy out
  // of the virtual owner's scratch slab)
  int ship(int64_t k, int64_t b0, int64_t b1, void* rccl, hipStream_t s) const {
    b1 = std::min(b1, nb);
    if (b1 <= b0) return GELIM_OK;
    double* c = col(k) + (b0 - k) * NB * NB;
    const int64_t n = (b1 - b0) * NB * NB;
    if (a.replay && !owns(k)) {
      HIP_TRY(hipMemcpyAsync(c, a.F[k % 3] + b0 * NB * NB, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    } else if (rccl) {
      GELIM_TRY(gelim_rccl_bcast(rccl, c, n, 0, (int)(k % a.P), s));
    }
    return GELIM_OK;
  }
  // A receiver's landing buffer X[t % 3] held column t-3: the side stream
  // (panel t-3), main (chain step t-3 reads it) and comm (its step t-3 reads
  // it; that step ends with kBulk(t-2)) must be done with it
  int land(int64_t t, hipStream_t s, bool on_main) const {
    if (owns(t) || t < 3) return GELIM_OK;
    HIP_TRY(hipStreamWaitEvent(s, ev(t - 3, kRest), 0));
    HIP_TRY(hipStreamWaitEvent(s, on_main ? ev(t - 2, kBulk) : ev(t - 3, kW), 0));
    return GELIM_OK;
  }
  // small_t = [Dinv_t; L_{t+1,t}], the chain message, on main
  int ship_small(int64_t t) {
    GELIM_TRY(land(t, main, true));
    GELIM_TRY(ship(t, t, t + 2, a.rccl_small, main));
    HIP_TRY(hipEventRecord(ev(t, kSmall), main));
    return GELIM_OK;
  }
  // next_t = L_{t+2,t} and rest_t = L_{t+3..,t} on comm; with f (the slab
  // of column t, owner's view) and k = t - 1, the rows they hold are first
  // updated there: f[t+2] -= L_{t+2,k} W, ship next, f[t+3..] -= L_{t+3..,k} W,
  // ship rest.  The rows beyond small_k come from next_k / rest_k, which
  // precede these on comm.
  int ship_below(int64_t t, double* f, const double* c, const double* W) {
    if (f && t + 2 < nb) GELIM_TRY(tile_gemm(f + (t + 2) * NB * NB, NB, c + 3 * NB * NB, NB, W, NB, NB, 1, comm));
    GELIM_TRY(land(t, comm, false));
    GELIM_TRY(ship(t, t + 2, t + 3, a.rccl_bulk, comm));
    HIP_TRY(hipEventRecord(ev(t, kNext), comm));
    if (f && t + 3 < nb)
      GELIM_TRY(gemm(f + (t + 3) * NB * NB, NB, 0, c + 4 * NB * NB, NB, W, NB, 0, (nb - t - 3) * NB, NB, NB, -1.0, 1,
                     a.side_cap, comm));
    GELIM_TRY(ship(t, t + 3, nb, a.rccl_bulk, comm));
    HIP_TRY(hipEventRecord(ev(t, kBulk), comm));
    if (a.replay && !owns(t)) HIP_TRY(hipEventRecord(ev(t, kShipDone), comm));
    return GELIM_OK;
  }

  // The chain step that produces block t = k+1 on its slab f (ld 128, the
  // column from row 0).  Main: W = Dinv_k f[k]; f[t] -= L_{t,k} W (both from
  // small_k alone); Dinv_t = f[t]^-1 in place; ship small_t once comm has
  // updated f[t+1].  Comm, beside the inverse: f[t+1] -= L_{t+1,k} W (next_k),
  // then the rows below with their messages (ship_below).  So the chain is
  // small_k -> W -> diagonal -> inverse -> small_t, and neither it nor the
  // next-row product waits on the bulk of a column.
  // below: the event of the apply of panel k-1 to the whole of block t (the
  // caller made main wait for its top rows only)
  int chain(int64_t k, double* f, int32_t* info, hipEvent_t below) {
    const int64_t t = k + 1;
    const double* c = col(k);
    double* W = wbuf(k);
    if (k >= 2) HIP_TRY(hipStreamWaitEvent(main, ev(k - 1, kBulk), 0));  // comm's step k-2 is done with this W
    GELIM_TRY(tile_gemm(W, NB, c, NB, f + k * NB * NB, NB, NB, 0, main));
    GELIM_TRY(tile_gemm(f + t * NB * NB, NB, c + NB * NB, NB, W, NB, NB, 1, main));
    HIP_TRY(hipEventRecord(ev(k, kW), main));
    GELIM_TRY(invert(f + t * NB * NB, t * NB, info, main));
    HIP_TRY(hipStreamWaitEvent(comm, ev(k, kW), 0));
    if (below) HIP_TRY(hipStreamWaitEvent(comm, below, 0));
    if (t + 1 < nb) GELIM_TRY(tile_gemm(f + (t + 1) * NB * NB, NB, c + 2 * NB * NB, NB, W, NB, NB, 1, comm));
    HIP_TRY(hipEventRecord(ev(k, kNR), comm));
    GELIM_TRY(ship_below(t, f, c, W));
    HIP_TRY(hipStreamWaitEvent(main, ev(k, kNR), 0));
    return ship_small(t);
  }

  // replay: the virtual owner of block k+2 applies panel k to it first --
  // its top rows (what that owner's chain step reads on main) ...
  int foreign_top(int64_t k) {
    const int64_t t = k + 2;
    if (!a.replay || t >= nb || owns(t)) return GELIM_OK;
    double* f = a.F[t % 3];
    const double* c = col(k);
    double* W = a.Wfs + (k & 1) * NB * NB;  // a ring of two: foreign_rest(k - 1) still reads the other
    HIP_TRY(hipStreamWaitEvent(aux, ev(k, kSmall), 0));
    HIP_TRY(hipStreamWaitEvent(aux, ev(k, kNext), 0));
    if (t >= 3) HIP_TRY(hipStreamWaitEvent(aux, ev(t - 3, kShipDone), 0));  // the slab's previous column shipped
    GELIM_TRY(tile_gemm(W, NB, c, NB, f + k * NB * NB, NB, NB, 0, aux));
    const int64_t top = std::min<int64_t>(2, nb - k - 1);  // block rows k+1, k+2
    GELIM_TRY(tile_gemm(f + (k + 1) * NB * NB, NB, c + NB * NB, NB, W, NB, top * NB, 1, aux));
    HIP_TRY(hipEventRecord(ev(t, kAuxTop), aux));
    return GELIM_OK;
  }
  // ... and the rows below, once rest_k has landed.  Issued AFTER the next
  // step's foreign_top: on the real run these are different owners' side
  // streams, so one owner's top rows never queue behind another's bulk (a
  // single replay stream in plain step order serialised them)
  int foreign_rest(int64_t k) {
    const int64_t t = k + 2;
    if (!a.replay || t >= nb || owns(t)) return GELIM_OK;
    double* f = a.F[t % 3];
    const double* c = col(k);
    const double* W = a.Wfs + (k & 1) * NB * NB;
    const int64_t top = std::min<int64_t>(2, nb - k - 1);
    HIP_TRY(hipStreamWaitEvent(aux, ev(k, kBulk), 0));
    GELIM_TRY(gemm(f + (k + 1 + top) * NB * NB, NB, 0, c + (1 + top) * NB * NB, NB, W, NB, 0,
                   a.np - (k + 1 + top) * NB, NB, NB, -1.0, 1, a.side_cap, aux));
    HIP_TRY(hipEventRecord(ev(t, kAuxSide), aux));
    return GELIM_OK;
  }

  int run() {
    HIP_TRY(hipEventRecord(ev(0, kRest), main));  // Mb as the transform left it
    HIP_TRY(hipStreamWaitEvent(side, ev(0, kRest), 0));
    HIP_TRY(hipStreamWaitEvent(comm, ev(0, kRest), 0));
    if (a.rank == 0)
      GELIM_TRY(invert(a.Mb, 0, a.info, main));
    else if (a.replay)
      GELIM_TRY(invert(a.F[0], 0, a.finfo, main));
    GELIM_TRY(ship_small(0));
    GELIM_TRY(ship_below(0, nullptr, nullptr, nullptr));
    for (int64_t k = 0; k < nb; ++k) {
      const double* c = col(k);
      const int64_t t = k + 1, lb0 = first_lb_after(k);
      const bool nxt = t < nb;
      const bool mine1 = nxt && owns(t);
      // main first: the chain step of block k+1 depends only on the previous
      // steps' side / aux work, so it is queued before this step's
      if (mine1) {
        if (k >= 1) HIP_TRY(hipStreamWaitEvent(main, ev(k - 1, kTop), 0));  // panel k-1 reached block k+1's top
        GELIM_TRY(chain(k, a.Mb + lb0 * a.mbs, a.info, k >= 1 ? ev(k - 1, kFirst) : nullptr));
      } else if (nxt && a.replay) {  // the virtual owner of block k+1, on this GPU
        if (t >= 2) HIP_TRY(hipStreamWaitEvent(main, ev(t, kAuxTop), 0));
        GELIM_TRY(chain(k, a.F[t % 3], a.finfo, t >= 2 ? ev(t, kAuxSide) : nullptr));
      } else if (nxt) {
        GELIM_TRY(ship_small(t));
        HIP_TRY(hipEventRecord(ev(k, kW), main));
        GELIM_TRY(ship_below(t, nullptr, nullptr, nullptr));
      }
      HIP_TRY(hipStreamWaitEvent(side, ev(k, kSmall), 0));
      HIP_TRY(hipStreamWaitEvent(side, ev(k, kNext), 0));
      const int64_t ls = lb0 + (mine1 ? 1 : 0);  // block k+1 is main's
      const int64_t lf = std::min(ls + 1, nbl);
      GELIM_TRY(apply_panel(k, c, ls, lf, a.Ws, a.nloc, a.side_cap, side, ev(k, kTop)));
      HIP_TRY(hipEventRecord(ev(k, kFirst), side));
      GELIM_TRY(apply_panel(k, c, lf, nbl, a.Ws + (lf - ls) * NB, a.nloc, a.side_cap, side));
      HIP_TRY(hipEventRecord(ev(k, kRest), side));
      GELIM_TRY(foreign_top(k));
      if (k >= 1) GELIM_TRY(foreign_rest(k - 1));
    }
    GELIM_TRY(foreign_rest(nb - 1));
    HIP_TRY(hipStreamWaitEvent(main, ev(nb - 1, kRest), 0));
    HIP_TRY(hipStreamWaitEvent(main, ev(nb - 1, kBulk), 0));
    if (a.replay) {
      HIP_TRY(hipEventRecord(ev(0, kAuxSide), aux));
      HIP_TRY(hipStreamWaitEvent(main, ev(0, kAuxSide), 0));
    }
    return GELIM_OK;
  }
};

}  // namespace

// The chain step's small products alone (tests and micro-benchmarks):
// with_w = 1: W = Dk B, then D -= L W; with_w = 0: D -= L W (W given).
// Every operand is 128 x 128, row-major, ld 128.
extern "C" int gelim_drbt_chain_products(const double* Dk, const double* B, double* W, const double* L, double* D,
                                         int32_t with_w, void* stream) {
  if (!W || !L || !D || (with_w && (!Dk || !B))) return GELIM_FAIL(GELIM_E_ARG, "drbt_chain_products: null operand");
  if (with_w) GELIM_TRY(tile_gemm(W, NB, Dk, NB, B, NB, NB, 0, (hipStream_t)stream));
  return tile_gemm(D, NB, L, NB, W, NB, NB, 1, (hipStream_t)stream);
}

// sizeof / offsetof of the argument block, for the Python mirror's layout test
// (tests/test_dist_rbt_cpu.py): which = 0 size, 1 offset of Wm, 2 of side_cap,
// 3 of Wfs, 4 of finfo.
extern "C" int64_t gelim_drbt_args_layout(int32_t which) {
  switch (which) {
    case 0: return (int64_t)sizeof(gelim_drbt_args);
    case 1: return (int64_t)offsetof(gelim_drbt_args, Wm);
    case 2: return (int64_t)offsetof(gelim_drbt_args, side_cap);
    case 3: return (int64_t)offsetof(gelim_drbt_args, Wfs);
    case 4: return (int64_t)offsetof(gelim_drbt_args, finfo);
    default: return -1;
  }
}

// The grid cap (CUs) of the bulk GEMMs beside the chain: all CUs but 16,
// which the chain's inverse and tile products then always find free
// (parallel/dist_rbt.py side_cap; one-rank-of-8 replay, four alternating
// rounds on one box: factor 6.8-7.1 ms at CUs - 16 in 4 of 4 processes,
// 7.0-8.4 at CUs - 32, 6.9-8.5 uncapped; another box ran 7.1-8.3 at every
// cap, profiles/dist_rbt_replay_r6.md).
extern "C" int gelim_drbt_side_cap(void) {
  int dev = 0, ncu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return ncu > 64 ? ncu - 16 : 0;
}

extern "C" gelim_drbt_exec* gelim_drbt_exec_create(void) { return new gelim_drbt_exec(); }

extern "C" void gelim_drbt_exec_destroy(gelim_drbt_exec* ex) {
  if (!ex) return;
  for (hipEvent_t e : ex->ev) (void)hipEventDestroy(e);
  delete ex;
}

// Issue the whole lookahead factorisation (asynchronous: returns once the
// work is queued; main then waits for every stream's last work).
extern "C" int gelim_drbt_factor(gelim_drbt_exec* ex, const gelim_drbt_args* a) {
  if (!ex || !a || !a->Mb || !a->Wm || !a->Ws || !a->info || a->P < 1 || a->rank < 0 || a->rank >= a->P ||
      a->np % (512 * (int64_t)a->P) || a->nloc * a->P != a->np || a->mbs < a->np * NB || !a->side ||
      !a->comm || (a->P > 1 && !a->replay && (!a->rccl_small || !a->rccl_bulk)) ||
      (a->replay && (!a->aux || !a->F[0] || !a->F[1] || !a->F[2] || !a->Wfs || !a->finfo)) ||
      !a->X[0] || !a->X[1] || !a->X[2])
    return GELIM_FAIL(GELIM_E_ARG, "drbt_factor: bad arguments");
  const int64_t nb = a->np / NB;
  GELIM_TRY(mk_events(ex, (int)nb));
  Exec e{*a, ex, (hipStream_t)a->main, (hipStream_t)a->side, (hipStream_t)a->comm, (hipStream_t)a->aux, nb,
         a->nloc / NB};
  return e.run();
}
