// Shared plumbing for the command-line front ends (L5 of SURVEY.md §1):
// backend names, timers, JSON result lines, the GPU solve path.
#pragma once

#include <hip/hip_runtime.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gelim/gelim.h"

namespace cli {

enum Backend { SEQ, OMP, PTH_V1, PTH_V2, PTH_V3, HIP_BLOCKED, HIP_PIVOT };

inline bool parse_backend(const char* s, Backend* b) {
  struct {
    const char* name;
    Backend b;
  } tab[] = {{"seq", SEQ},           {"omp", OMP},
             {"openmp", OMP},        {"pthreads-v1", PTH_V1},
             {"pthreads-v2", PTH_V2}, {"pthreads-v3", PTH_V3},
             {"hip", HIP_BLOCKED},   {"hip-blocked", HIP_BLOCKED},
             {"hip-pivot", HIP_PIVOT}};
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
  }
  return "?";
}

inline bool is_gpu(Backend b) { return b == HIP_BLOCKED || b == HIP_PIVOT; }

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

}  // namespace cli
