// Shared plumbing for the command-line front ends (L5 of SURVEY.md §1):
// backend names, timers, JSON result lines, the GPU solve path.
#pragma once

#include <hip/hip_runtime.h>
#include <sys/time.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gelim/gelim.h"

namespace cli {

enum Backend { SEQ, OMP, PTH_V1, PTH_V2, PTH_V3, HIP_BLOCKED, HIP_PIVOT, HIP_RBT };

inline bool parse_backend(const char* s, Backend* b) {
  struct {
    const char* name;
    Backend b;
  } tab[] = {{"seq", SEQ},           {"omp", OMP},
             {"openmp", OMP},        {"pthreads-v1", PTH_V1},
             {"pthreads-v2", PTH_V2}, {"pthreads-v3", PTH_V3},
             {"hip", HIP_BLOCKED},   {"hip-blocked", HIP_BLOCKED},
             {"hip-pivot", HIP_PIVOT},   {"hip-rbt", HIP_RBT}};
  for (auto& e : tab)
    if (std::strcmp(s, e.name) == 0) {
      *b = e.b;
      return true;
    }
  return false;
}

inline const char* backend_name(Backend b) {
  switch (b) {
    case SEQ: return "seq";
    case OMP: return "omp";
    case PTH_V1: return "pthreads-v1";
    case PTH_V2: return "pthreads-v2";
    case PTH_V3: return "pthreads-v3";
    case HIP_BLOCKED: return "hip-blocked";
    case HIP_PIVOT: return "hip-pivot";
    case HIP_RBT: return "hip-rbt";
  }
  return "?";
}

inline bool is_gpu(Backend b) { return b == HIP_BLOCKED || b == HIP_PIVOT || b == HIP_RBT; }

inline int cpu_backend_code(Backend b) {
  switch (b) {
    case SEQ: return GELIM_CPU_SEQ;
    case OMP: return GELIM_CPU_OMP;
    case PTH_V1: return GELIM_CPU_PTH_V1;
    case PTH_V2: return GELIM_CPU_PTH_V2;
    default: return GELIM_CPU_PTH_V3;
  }
}

// gettimeofday, like the reference timers (P1i:278-290).
inline double wall() {
  struct timeval tv;
  gettimeofday(&tv, nullptr);
  return (double)tv.tv_sec + (double)tv.tv_usec * 1e-6;
}

inline std::string device_name() {
  hipDeviceProp_t prop;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess)
    return "unknown";
  return std::string(prop.name) + " (" + prop.gcnArchName + ")";
}

[[noreturn]] inline void die(const char* what) {
  std::fprintf(stderr, "%s: %s\n", what, gelim_last_error());
  std::exit(-1);
}

// A GPU backend on a host without a HIP device: say so (and what to use
// instead) before any HIP call fails with a runtime message.
inline void require_gpu(const char* what, const char* instead) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    std::fprintf(stderr, "no HIP device found: %s needs an AMD GPU; %s\n", what, instead);
    std::exit(-1);
  }
}

#define CLI_CHECK(expr)                 \
  do {                                  \
    if ((expr) != 0) cli::die(#expr);   \
  } while (0)

#define CLI_HIP(expr)                                                              \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d: %s: %s\n", __FILE__, __LINE__, #expr,           \
                   hipGetErrorString(_e));                                         \
      std::exit(-1);                                                               \
    }                                                                              \
  } while (0)

// hip-rbt: the randomised no-pivoting fp64 engine (random butterfly transform
// + block LDU on the matrix cores + fp64 refinement to a componentwise
// backward error <= 4 eps, csrc/hip/lu_mixed.hip) on a device augmented
// system; when the engine asks for it (zero pivot / stalled refinement) the
// same system goes to the blocked LU with the reference's pivoting rule.
struct RbtSolver {
  int64_t n;
  int pivot;
  bool use_graph;
  gelim_mixed_plan* plan = nullptr;
  gelim_gauss_plan* fallback = nullptr;
  bool fell_back = false;
  int steps = 0;
  double berr = 0.0;

  RbtSolver(int64_t n_, int pivot_, bool graph) : n(n_), pivot(pivot_), use_graph(graph) {
    const int64_t np = gelim_mixed_padded(n);
    std::vector<double> ud(2 * np), vd(2 * np);
    uint64_t st = 0x5eedull;  // splitmix64: a fixed, platform-independent butterfly
    auto uni = [&st]() {
      uint64_t z = (st += 0x9e3779b97f4a7c15ull);
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      return (double)((z ^ (z >> 31)) >> 11) * 0x1.0p-53;
    };
    for (auto& v : ud) v = std::exp((uni() - 0.5) / 10.0);
    for (auto& v : vd) v = std::exp((uni() - 0.5) / 10.0);
    plan = gelim_mixed_plan_create2(n, ud.data(), vd.data(), 1);
    if (!plan) die("mixed_plan_create");
  }
  ~RbtSolver() {
    if (plan) gelim_mixed_plan_destroy(plan);
    if (fallback) gelim_gauss_plan_destroy(fallback);
  }
  void solve(const double* d_aug, int64_t ld, double* d_x, hipStream_t s) {
    const int rc = gelim_mixed_solve(plan, d_aug, ld, d_x, 6, &steps, &berr, s);
    if (rc < 0) die("mixed_solve");
    fell_back = rc == 1;
    if (fell_back) {
      if (!fallback) fallback = gelim_gauss_plan_create(n, GELIM_GPU_BLOCKED, pivot, 8, use_graph);
      if (!fallback) die("plan_create");
      if (gelim_gauss_plan_solve(fallback, d_aug, ld, d_x, nullptr, s) != 0) die("plan_solve");
    }
  }
  // 0, or 1 + the first zero-pivot column (only the fallback can tell)
  int info(hipStream_t s) { return fell_back ? gelim_gauss_plan_info(fallback, s) : 0; }
  void note() const {
    std::printf("hip-rbt: %d corrections, componentwise backward error %.3e%s\n", steps, berr,
                fell_back ? " -> fell back to partial pivoting" : "");
  }
};

}  // namespace cli
