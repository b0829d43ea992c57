// CPU reference backends for Gaussian elimination (L2/L3 of SURVEY.md §1).
//
// One implementation of the numerical core (N6-N10) shared by five parallel
// strategies:
//   SEQ     sequential, the exact reference loop order
//           (OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182)
//   OMP     `omp parallel for` over the rows below the pivot (S4)
//   PTH_V1  pthreads fork-join, rows cyclic, T threads created per pivot (S1,
//           Pthreads/Version-1/gauss_internal_input.c:140-206)
//   PTH_V2  as V1 with 16-column strips so the pivot-row strip stays in cache
//           (S2, Pthreads/Version-2/gauss_internal_input.c:142-216)
//   PTH_V3  persistent threads; thread 0 pivots, a barrier separates steps,
//           optional CPU pinning (S3, Pthreads/Version-3/gauss_internal_input.c:150-202).
//           Unlike the reference the barrier is a generation-counted
//           mutex/condvar barrier with a predicate loop (the reference's is
//           racy) and thread state is sized after `-t` is
//           parsed (the reference overflows for -t > 32, §2.8-1).
// Every backend performs the same floating-point operations per row in the
// same order, so all of them produce bit-identical results (the reference
// observed identical `Error:` values across backends).
#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "gelim/internal.h"

namespace {

constexpr int kBlockSize = 16;  // V2 column strip (P2i:18)

struct System {
  double* A;
  int64_t lda;
  double* b;
  int64_t n;
  double* row(int64_t i) const { return A + i * lda; }
};

// Pivot selection + row swap + pivot-row normalisation for step i.
// Returns false if the matrix is singular at this step.
bool pivot_step(const System& s, int64_t i, int mode) {
  const int64_t n = s.n;
  int64_t prow = i;
  if (mode == GELIM_PIVOT_PARTIAL) {
    // argmax |A[r][i]|, strict '>' so ties keep the lowest row (P1e:130-134)
    double best = std::fabs(s.row(i)[i]);
    for (int64_t r = i + 1; r < n; ++r) {
      double v = std::fabs(s.row(r)[i]);
      if (v > best) {
        best = v;
        prow = r;
      }
    }
    if (best == 0.0) return false;
  } else {
    // swap only if the diagonal is exactly zero (P1i:84-98)
    if (s.row(i)[i] == 0.0) {
      prow = -1;
      for (int64_t r = i; r < n; ++r)
        if (s.row(r)[i] != 0.0) {
          prow = r;
          break;
        }
      if (prow < 0) return false;
    }
  }
  if (prow != i) {
    double* a = s.row(i);
    double* c = s.row(prow);
    for (int64_t k = i; k < n; ++k) std::swap(a[k], c[k]);
    std::swap(s.b[i], s.b[prow]);
  }
  // Normalise the pivot row to a unit diagonal (P1i:109-120, P1e:219-227).
  double* a = s.row(i);
  double p = a[i];
  if (p != 1.0) {
    a[i] = 1.0;
    for (int64_t k = i + 1; k < n; ++k) a[k] /= p;
    s.b[i] /= p;
  }
  return true;
}

// Eliminate one row j below pivot i (N9).
inline void eliminate_row(const System& s, int64_t i, int64_t j) {
  double* aj = s.row(j);
  const double* ai = s.row(i);
  const double m = aj[i];
  aj[i] = 0.0;
  for (int64_t k = i + 1; k < s.n; ++k) aj[k] -= m * ai[k];
  s.b[j] -= m * s.b[i];
}

// V2: strip-blocked elimination of the rows owned by thread `tid` (cyclic).
void eliminate_rows_blocked(const System& s, int64_t i, int tid, int T) {
  const int64_t n = s.n;
  const double* ai = s.row(i);
  for (int64_t j = i + 1 + tid; j < n; j += T) s.b[j] -= s.row(j)[i] * s.b[i];
  for (int64_t k0 = i + 1; k0 < n; k0 += kBlockSize) {
    const int64_t k1 = std::min<int64_t>(k0 + kBlockSize, n);
    for (int64_t j = i + 1 + tid; j < n; j += T) {
      double* aj = s.row(j);
      const double m = aj[i];
      for (int64_t k = k0; k < k1; ++k) aj[k] -= m * ai[k];
    }
  }
  for (int64_t j = i + 1 + tid; j < n; j += T) s.row(j)[i] = 0.0;
}

int singular(int64_t i) {
  return GELIM_FAIL(GELIM_E_SINGULAR,
                    "The matrix is singular (zero pivot at column " + std::to_string(i) + ")");
}

int run_seq(const System& s, int mode) {
  for (int64_t i = 0; i < s.n; ++i) {
    if (!pivot_step(s, i, mode)) return singular(i);
    for (int64_t j = i + 1; j < s.n; ++j) eliminate_row(s, i, j);
  }
  return GELIM_OK;
}

int run_omp(const System& s, int mode, int threads) {
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
  for (int64_t i = 0; i < s.n; ++i) {
    if (!pivot_step(s, i, mode)) return singular(i);
#pragma omp parallel for schedule(static)
    for (int64_t j = i + 1; j < s.n; ++j) eliminate_row(s, i, j);
  }
  return GELIM_OK;
}

struct ForkJoinArgs {
  const System* s;
  int64_t i;
  int tid, T;
  bool blocked;
};

void* fork_join_worker(void* p) {
  auto* a = static_cast<ForkJoinArgs*>(p);
  if (a->blocked) {
    eliminate_rows_blocked(*a->s, a->i, a->tid, a->T);
  } else {
    for (int64_t j = a->i + 1 + a->tid; j < a->s->n; j += a->T) eliminate_row(*a->s, a->i, j);
  }
  return nullptr;
}

int run_fork_join(const System& s, int mode, int T, bool blocked) {
  std::vector<pthread_t> th(T);
  std::vector<ForkJoinArgs> args(T);
  for (int64_t i = 0; i < s.n; ++i) {
    if (!pivot_step(s, i, mode)) return singular(i);
    for (int t = 0; t < T; ++t) {
      args[t] = {&s, i, t, T, blocked};
      int rc = pthread_create(&th[t], nullptr, fork_join_worker, &args[t]);
      if (rc) {
        for (int u = 0; u < t; ++u) pthread_join(th[u], nullptr);
        return GELIM_FAIL(GELIM_E_THREAD,
                          "ERROR; return code from pthread_create() is " + std::to_string(rc));
      }
    }
    for (int t = 0; t < T; ++t) pthread_join(th[t], nullptr);
  }
  return GELIM_OK;
}

// Generation-counted barrier (fixes the reference V3 barrier race).
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(m_);
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

struct PersistentShared {
  const System* s;
  int mode, T;
  Barrier barrier;
  int64_t failed_at = -1;
  PersistentShared(const System* s_, int m, int t) : s(s_), mode(m), T(t), barrier(t) {}
};

struct PersistentArgs {
  PersistentShared* sh;
  int tid;
};

void* persistent_worker(void* p) {
  auto* a = static_cast<PersistentArgs*>(p);
  PersistentShared& sh = *a->sh;
  const System& s = *sh.s;
  for (int64_t i = 0; i < s.n; ++i) {
    // Thread 0 alone pivots (P3i:162-174); the barrier publishes its writes.
    if (a->tid == 0 && sh.failed_at < 0 && !pivot_step(s, i, sh.mode)) sh.failed_at = i;
    sh.barrier.arrive_and_wait();
    if (sh.failed_at >= 0) return nullptr;  // every thread sees it after the barrier
    for (int64_t j = i + 1 + a->tid; j < s.n; j += sh.T) eliminate_row(s, i, j);
    sh.barrier.arrive_and_wait();  // row updates done before the next pivot
  }
  return nullptr;
}

int run_persistent(const System& s, int mode, int T, int affinity) {
  PersistentShared sh(&s, mode, T);
  std::vector<pthread_t> th(T);
  std::vector<PersistentArgs> args(T);
  const long nprocs = sysconf(_SC_NPROCESSORS_ONLN);
  const bool pin = affinity && T <= nprocs;  // P3i:278-283
  for (int t = 0; t < T; ++t) {
    args[t] = {&sh, t};
    pthread_attr_t attr;
    pthread_attr_init(&attr);
    if (pin) {
      cpu_set_t cs;
      CPU_ZERO(&cs);
      CPU_SET(t, &cs);
      pthread_attr_setaffinity_np(&attr, sizeof cs, &cs);
    }
    int rc = pthread_create(&th[t], &attr, persistent_worker, &args[t]);
    pthread_attr_destroy(&attr);
    if (rc) {
      // Threads already started would wait forever on the barrier; this path
      // aborts the process like the reference (exit(-1)).
      std::fprintf(stderr, "ERROR; return code from pthread_create() is %d\n", rc);
      std::exit(-1);
    }
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], nullptr);
  if (sh.failed_at >= 0) return singular(sh.failed_at);
  return GELIM_OK;
}

}  // namespace

extern "C" int gelim_cpu_gauss(double* A, int64_t lda, double* b, int64_t n,
                               int pivot, int backend, int threads,
                               int affinity) {
  if (!A || !b || n <= 0 || lda < n) return GELIM_FAIL(GELIM_E_ARG, "bad gauss args");
  if (pivot != GELIM_PIVOT_ZERO && pivot != GELIM_PIVOT_PARTIAL)
    return GELIM_FAIL(GELIM_E_ARG, "bad pivot mode");
  System s{A, lda, b, n};
  const int T = threads > 0 ? threads : 32;  // default num_threads = 32 (P1i:25)
  switch (backend) {
    case GELIM_CPU_SEQ: return run_seq(s, pivot);
    case GELIM_CPU_OMP: return run_omp(s, pivot, threads);
    case GELIM_CPU_PTH_V1: return run_fork_join(s, pivot, T, false);
    case GELIM_CPU_PTH_V2: return run_fork_join(s, pivot, T, true);
    case GELIM_CPU_PTH_V3:
      if (T < 2) return GELIM_FAIL(GELIM_E_ARG, "V3 needs at least 2 threads");
      return run_persistent(s, pivot, T, affinity);
    default: return GELIM_FAIL(GELIM_E_ARG, "unknown CPU backend");
  }
}

extern "C" int gelim_cpu_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return (int)sysconf(_SC_NPROCESSORS_ONLN);
#endif
}

extern "C" void gelim_cpu_backsub_unit(const double* U, int64_t ldu,
                                       const double* b, double* x, int64_t n) {
  // N10: V[n-1] = B[n-1]; V[i] = B[i] - sum_{j>i} U[i][j] V[j], j descending.
  x[n - 1] = b[n - 1];
  for (int64_t i = n - 2; i >= 0; --i) {
    double v = b[i];
    const double* row = U + i * ldu;
    for (int64_t j = n - 1; j > i; --j) v -= row[j] * x[j];
    x[i] = v;
  }
}

// ---------------------------------------------------------------------------
// Blocked-LU building blocks (CPU versions of the HIP kernels; used by the
// distributed driver when ranks run on CPU with gloo, and as test oracles).
// ---------------------------------------------------------------------------

extern "C" int gelim_cpu_panel_factor(double* P, int64_t ldp, int64_t m,
                                      int64_t w, int64_t row0, int pivot,
                                      int32_t* piv, int32_t* info) {
  if (!P || m <= 0 || w <= 0 || w > m || ldp < w) return GELIM_FAIL(GELIM_E_ARG, "bad panel args");
  for (int64_t j = 0; j < w; ++j) {
    int64_t p = j;
    if (pivot == GELIM_PIVOT_PARTIAL) {
      double best = std::fabs(P[j * ldp + j]);
      for (int64_t r = j + 1; r < m; ++r) {
        double v = std::fabs(P[r * ldp + j]);
        if (v > best) {
          best = v;
          p = r;
        }
      }
    } else if (P[j * ldp + j] == 0.0) {
      for (int64_t r = j + 1; r < m; ++r)
        if (P[r * ldp + j] != 0.0) {
          p = r;
          break;
        }
    }
    piv[j] = (int32_t)p;
    if (p != j)
      for (int64_t c = 0; c < w; ++c) std::swap(P[j * ldp + c], P[p * ldp + c]);
    const double d = P[j * ldp + j];
    if (d == 0.0) {
      if (info && *info == 0) *info = (int32_t)(row0 + j + 1);
      continue;
    }
    const double rd = 1.0 / d;
    for (int64_t r = j + 1; r < m; ++r) {
      double* pr = P + r * ldp;
      const double l = pr[j] * rd;
      pr[j] = l;
      for (int64_t c = j + 1; c < w; ++c) pr[c] -= l * P[j * ldp + c];
    }
  }
  return GELIM_OK;
}

extern "C" int gelim_cpu_swap_trsm(double* C, int64_t ldc, int64_t ncols,
                                   const double* L, int64_t ldl, int64_t w,
                                   const int32_t* piv, int64_t row0,
                                   int64_t nrows) {
  (void)row0;
  if (ncols <= 0) return GELIM_OK;
  for (int64_t j = 0; j < w; ++j) {
    const int64_t p = piv[j];
    if (p < 0 || p >= nrows) return GELIM_FAIL(GELIM_E_ARG, "pivot out of range");
    if (p != j)
      for (int64_t c = 0; c < ncols; ++c) std::swap(C[j * ldc + c], C[p * ldc + c]);
  }
  for (int64_t j = 1; j < w; ++j)
    for (int64_t i = 0; i < j; ++i) {
      const double l = L[j * ldl + i];
      for (int64_t c = 0; c < ncols; ++c) C[j * ldc + c] -= l * C[i * ldc + c];
    }
  return GELIM_OK;
}

extern "C" int gelim_cpu_gemm_update(double* C, int64_t ldc, const double* L,
                                     int64_t ldl, const double* U, int64_t ldu,
                                     int64_t M, int64_t N, int64_t K) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < M; ++i)
    for (int64_t k = 0; k < K; ++k) {
      const double l = L[i * ldl + k];
      const double* u = U + k * ldu;
      double* c = C + i * ldc;
      for (int64_t j = 0; j < N; ++j) c[j] -= l * u[j];
    }
  return GELIM_OK;
}
