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
// Per block k (owner o = k % P), messages [Dinv_k; L_{k+1,k}] ("small",
// the chain's) and L_{k+2..,k} ("bulk"):
//   small: on the MAIN stream through its own communicator -- the chain
//          (wait small -> W -> diagonal update -> inverse -> column rest ->
//          next small) then has no cross-stream hop besides the bulk's;
//   bulk:  on the COMM stream through a second communicator, so it travels
//          under the chain and never delays the next small message.
// Owner of k+1, main: W = Dinv_k M[k, k+1]; M[k+1,k+1] -= L_{k+1,k} W;
//   Dinv_{k+1} in place; [bulk_k] M[k+2..,k+1] -= L_{k+2..,k} W; ship k+1.
// Every rank, side: [small_k, bulk_k] panel k -> its next block (ev_first),
//   then the rest of its columns (ev_rest).
// The GEMMs and inverses are the Python schedule's, with the same operands
// and shapes, so both give the same factor bits
// (tests/test_gpu_dist_rbt.py::test_native_executor_matches_python).
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
#include <cstdint>
#include <vector>

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
  double* Wm;           // 128 x 128 (main)
  double* Ws;           // 128 x nloc (side)
  int32_t* info;        // device: 1 + first column of a non-finite inverse (atomicMin)
  void* main;           // hipStream_t (null: the default stream)
  void* side;
  void* comm;
  void* rccl_small;     // communicators (null: no collective -- one rank, or the replay)
  void* rccl_bulk;
  int32_t side_cap;     // CUs for the side stream's bulk GEMMs (0 = all)
  int32_t replay;       // 1: replay mode (module comment)
  double* F[3];         // replay: scratch slabs np x 128
  void* aux;            // replay: the virtual owners' side stream
  double* Wf;           // replay: 128 x 128 (main) and 128 x 128 (aux)
  double* Wfs;
  int32_t* finfo;       // replay: the scratch inverses' info word
};

struct gelim_drbt_exec {
  int nb = 0;
  std::vector<hipEvent_t> ev;  // 7 per block
};

namespace {

constexpr int NB = 128;
enum { kSmall, kBulk, kShip, kFirst, kRest, kAuxSide, kShipDone, kNev };

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

  hipEvent_t ev(int k, int which) const { return ex->ev[(size_t)k * kNev + which]; }
  bool owns(int64_t k) const { return k % a.P == a.rank; }
  double* col(int64_t k) const {  // column k from its diagonal block down (ld 128)
    return owns(k) ? a.Mb + (k / a.P) * a.mbs + k * NB * NB : a.X[k % 3];
  }
  int64_t small(int64_t k) const { return std::min<int64_t>(2 * NB, a.np - k * NB); }
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
  int apply_panel(int64_t k, const double* c, int64_t lb0, int64_t lb1, double* W, int64_t ldw, int cap,
                  hipStream_t s) const {
    if (lb1 <= lb0) return GELIM_OK;
    GELIM_TRY(panel_w(k, c, lb0, lb1, W, ldw, s));
    return panel_rows(k, c, lb0, lb1, (k + 1) * NB, a.np, W, ldw, cap, s);
  }
  int invert(double* blk, int64_t colidx, int32_t* info, hipStream_t s) const {
    return gelim_rbt_block_inverse(blk, NB, colidx, blk, info, s);
  }

  // the chain message of block k, [Dinv_k; L_{k+1,k}], on the main stream
  // (the owner's slab in place; receivers into their landing buffer)
  int ship_small(int64_t k) {
    double* c = col(k);
    const int64_t sm = small(k) * NB;
    if (a.replay && !owns(k)) {
      HIP_TRY(hipMemcpyAsync(c, a.F[k % 3] + k * NB * NB, sm * sizeof(double), hipMemcpyDeviceToDevice, main));
    } else if (a.rccl_small) {
      GELIM_TRY(gelim_rccl_bcast(a.rccl_small, c, sm, 0, (int)(k % a.P), main));
    }
    HIP_TRY(hipEventRecord(ev(k, kSmall), main));
    return GELIM_OK;
  }
  // the rest of column k, L_{k+2..,k}, on the communicator stream after
  // what main has produced (owner) or freed (receivers) so far
  int ship_bulk(int64_t k) {
    double* c = col(k);
    const int64_t n = (a.np - k * NB) * NB, sm = small(k) * NB;
    HIP_TRY(hipEventRecord(ev(k, kShip), main));
    HIP_TRY(hipStreamWaitEvent(comm, ev(k, kShip), 0));
    if (n > sm) {
      if (a.replay && !owns(k)) {
        const double* src = a.F[k % 3] + k * NB * NB;
        HIP_TRY(hipMemcpyAsync(c + sm, src + sm, (n - sm) * sizeof(double), hipMemcpyDeviceToDevice, comm));
      } else if (a.rccl_bulk) {
        GELIM_TRY(gelim_rccl_bcast(a.rccl_bulk, c + sm, n - sm, 0, (int)(k % a.P), comm));
      }
    }
    HIP_TRY(hipEventRecord(ev(k, kBulk), comm));
    if (a.replay && !owns(k)) HIP_TRY(hipEventRecord(ev(k, kShipDone), comm));
    return GELIM_OK;
  }

  // The chain step that produces block t = k+1 on its slab f (ld 128, the
  // column from row 0): W = Dinv_k f[k]; f[t] -= L_{t,k} W; the next block
  // row f[t+1] -= L_{t+1,k} W (needs bulk_k's first block); Dinv_t = f[t]^-1
  // in place; ship small_t; the rest f[t+2..] -= L_{t+2..,k} W; ship bulk_t.
  // Only W, the diagonal update, the next-block row and the inverse are on
  // the chain: the next owner needs nothing else.
  int chain(int64_t k, double* f, int64_t fbs, double* W, int32_t* info) {
    const int64_t t = k + 1;
    const double* c = col(k);
    GELIM_TRY(gemm(W, NB, 0, c, NB, f + k * NB * NB, NB, fbs, NB, NB, NB, 1.0, 0, 0, main));
    GELIM_TRY(gemm(f + t * NB * NB, NB, fbs, c + NB * NB, NB, W, NB, 0, NB, NB, NB, -1.0, 1, 0, main));
    const bool more = (t + 1) * NB < a.np;
    if (more) {
      HIP_TRY(hipStreamWaitEvent(main, ev(k, kBulk), 0));
      GELIM_TRY(gemm(f + (t + 1) * NB * NB, NB, fbs, c + 2 * NB * NB, NB, W, NB, 0, NB, NB, NB, -1.0, 1, 0, main));
    }
    GELIM_TRY(invert(f + t * NB * NB, t * NB, info, main));
    // a receiver's landing buffer of t is free once its side stream is done with t - 3
    if (t >= 3 && !owns(t)) HIP_TRY(hipStreamWaitEvent(main, ev(t - 3, kRest), 0));
    GELIM_TRY(ship_small(t));
    if ((t + 2) * NB < a.np)
      GELIM_TRY(gemm(f + (t + 2) * NB * NB, NB, fbs, c + 3 * NB * NB, NB, W, NB, 0, a.np - (t + 2) * NB, NB, NB, -1.0,
                     1, 0, main));
    return ship_bulk(t);
  }

  // replay: the virtual owner of block k+2 applies panel k to it first
  int foreign_side(int64_t k) {
    const int64_t t = k + 2;
    if (!a.replay || t >= nb || owns(t)) return GELIM_OK;
    double* f = a.F[t % 3];
    const double* c = col(k);
    HIP_TRY(hipStreamWaitEvent(aux, ev(k, kSmall), 0));
    HIP_TRY(hipStreamWaitEvent(aux, ev(k, kBulk), 0));
    if (t >= 3) HIP_TRY(hipStreamWaitEvent(aux, ev(t - 3, kShipDone), 0));  // the slab's previous column shipped
    GELIM_TRY(gemm(a.Wfs, NB, 0, c, NB, f + k * NB * NB, NB, 0, NB, NB, NB, 1.0, 0, 0, aux));
    GELIM_TRY(gemm(f + (k + 1) * NB * NB, NB, 0, c + NB * NB, NB, a.Wfs, NB, 0, a.np - (k + 1) * NB, NB, NB, -1.0, 1,
                   a.side_cap, aux));
    HIP_TRY(hipEventRecord(ev(t, kAuxSide), aux));
    return GELIM_OK;
  }

  // replay: the virtual owner of block k+1 (k = -1: block 0's inverse)
  int foreign_chain(int64_t k) {
    const int64_t t = k + 1;
    double* f = a.F[t % 3];
    if (k < 0) return invert(f, 0, a.finfo, main);
    if (t >= 2) HIP_TRY(hipStreamWaitEvent(main, ev(t, kAuxSide), 0));
    return chain(k, f, 0, a.Wf, a.finfo);
  }

  int run() {
    HIP_TRY(hipEventRecord(ev(0, kRest), main));  // Mb as the transform left it
    HIP_TRY(hipStreamWaitEvent(side, ev(0, kRest), 0));
    if (a.rank == 0)
      GELIM_TRY(invert(a.Mb, 0, a.info, main));
    else if (a.replay)
      GELIM_TRY(foreign_chain(-1));
    GELIM_TRY(ship_small(0));
    GELIM_TRY(ship_bulk(0));
    for (int64_t k = 0; k < nb; ++k) {
      const double* c = col(k);
      const int64_t lb0 = first_lb_after(k);
      const bool nxt = k + 1 < nb;
      const bool mine1 = nxt && owns(k + 1);
      // main first: the chain step of block k+1 depends only on the previous
      // steps' side / aux work, so it is queued before this step's
      if (mine1) {
        if (k >= 1) HIP_TRY(hipStreamWaitEvent(main, ev(k - 1, kFirst), 0));  // panel k-1 reached block k+1
        GELIM_TRY(chain(k, a.Mb + lb0 * a.mbs, a.mbs, a.Wm, a.info));
      } else if (nxt && a.replay) {
        GELIM_TRY(foreign_chain(k));
      } else if (nxt) {
        if (k + 1 >= 3) HIP_TRY(hipStreamWaitEvent(main, ev(k + 1 - 3, kRest), 0));  // landing buffer free again
        GELIM_TRY(ship_small(k + 1));
        GELIM_TRY(ship_bulk(k + 1));
      }
      HIP_TRY(hipStreamWaitEvent(side, ev(k, kSmall), 0));
      HIP_TRY(hipStreamWaitEvent(side, ev(k, kBulk), 0));
      const int64_t ls = lb0 + (mine1 ? 1 : 0);  // block k+1 is main's
      const int64_t lf = std::min(ls + 1, nbl);
      GELIM_TRY(apply_panel(k, c, ls, lf, a.Ws, a.nloc, a.side_cap, side));
      HIP_TRY(hipEventRecord(ev(k, kFirst), side));
      GELIM_TRY(apply_panel(k, c, lf, nbl, a.Ws + (lf - ls) * NB, a.nloc, a.side_cap, side));
      HIP_TRY(hipEventRecord(ev(k, kRest), side));
      GELIM_TRY(foreign_side(k));
    }
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
      (a->replay && (!a->aux || !a->F[0] || !a->F[1] || !a->F[2] || !a->Wf || !a->Wfs || !a->finfo)) ||
      !a->X[0] || !a->X[1] || !a->X[2])
    return GELIM_FAIL(GELIM_E_ARG, "drbt_factor: bad arguments");
  const int64_t nb = a->np / NB;
  GELIM_TRY(mk_events(ex, (int)nb));
  Exec e{*a, ex, (hipStream_t)a->main, (hipStream_t)a->side, (hipStream_t)a->comm, (hipStream_t)a->aux, nb,
         a->nloc / NB};
  return e.run();
}
