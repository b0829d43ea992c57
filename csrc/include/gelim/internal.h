// Internal helpers shared by the host-side C++ and HIP translation units.
#pragma once

#include <cstdint>
#include <cstdio>
#include <string>

#include "gelim/gelim.h"

namespace gelim {

// Thread-local error message behind gelim_last_error().
void set_error(const std::string& msg);
int fail(int code, const char* file, int line, const std::string& msg);
// Zero `bytes` (a multiple of 4) of device memory with a kernel.  Used in
// place of hipMemsetAsync everywhere a solve may be graph-captured: memset
// nodes of captured graphs were the part of a graph that plan lifecycle
// operations corrupted on ROCm 7.2 (profiles/graph_recapture.txt).
int zero_async(void* p, size_t bytes, struct ihipStream_t* s);
// A non-blocking stream probed to run concurrently with the default stream
// (runtime.hip: streams sharing its hardware queue are parked, up to 8 tries).
int side_stream_create(struct ihipStream_t** out);
// Co-residency guard of the persistent (flag hand-off) kernels: true when
// `grid` workgroups of a kernel that the occupancy API admits `per_cu` times
// per CU all fit at once (one block of margin per CU above one, as the API
// can overstate the SGPR-limited count by one); GELIM_FORCE_NONPERSISTENT=1
// forces false (tests of the fallback schedules).
bool coresident(int per_cu, int64_t grid);
// Row-major 2D copy (rows x width bytes, width a multiple of 4) by a kernel,
// for the same reason (no memcpy nodes in captured graphs).
int copy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                 struct ihipStream_t* s);
// Up to kMaxFills word ranges set to a 32-bit pattern in ONE launch: a
// solve's prologue (status words, flag arrays, sentinel-filled outputs)
// without a launch per buffer.
struct WordFill {
  void* p;
  size_t bytes;  // a multiple of 4
  unsigned value;
};
constexpr int kMaxFills = 4;
// One row-major fp64 product C (M x N, ldc) += alpha A (M x K) B (K x N) of a
// grouped launch (dgemm.hip dgemm_pair: two independent products, one grid)
struct GemmOp {
  double* C;
  int64_t ldc;
  const double* A;
  int64_t lda;
  const double* B;
  int64_t ldb;
  int64_t M, N, K;
};
int dgemm_pair(const GemmOp& p1, const GemmOp& p2, double alpha, int accumulate, struct ihipStream_t* s);
// The same for K = 128 as 16 x 16 tiles, one 64-thread workgroup each, no LDS
// (dgemm.hip tile16_kernel): bit-identical to dgemm, for 128-wide products on
// a latency-bound chain.  M and N multiples of 16.
int dgemm_tiles(const GemmOp& p1, const GemmOp& p2, double alpha, int accumulate, struct ihipStream_t* s);
int fill_words_async(const WordFill* f, int nf, struct ihipStream_t* s);

}  // namespace gelim

#define GELIM_FAIL(code, msg) ::gelim::fail((code), __FILE__, __LINE__, (msg))

// Check a hipError_t; on failure record "file:line: hipGetErrorString" and
// return GELIM_E_HIP from the enclosing function (every HIP
// return code is checked — the reference never checks cudaError_t).
#define HIP_TRY(expr)                                                        \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess)                                                    \
      return ::gelim::fail(GELIM_E_HIP, __FILE__, __LINE__,                  \
                           std::string(#expr ": ") + hipGetErrorString(_e)); \
  } while (0)

#define GELIM_TRY(expr)      \
  do {                       \
    int _rc = (expr);        \
    if (_rc != 0) return _rc; \
  } while (0)
