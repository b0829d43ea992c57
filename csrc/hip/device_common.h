// Device-side helpers for the gfx950 kernels (wave64, CDNA4).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace gelim {
namespace dev {

constexpr int kWave = 64;  // CDNA wavefront width — never 32

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));

// (value, index) arg-max step: larger value wins, ties -> smaller index.
__device__ __forceinline__ void argmax_merge(double& v, int& i, double ov, int oi) {
  if (ov > v || (ov == v && oi < i)) {
    v = ov;
    i = oi;
  }
}

// Wave-wide arg-max over all 64 lanes; every lane gets the result.
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    double ov = __shfl_xor(v, off, kWave);
    int oi = __shfl_xor(i, off, kWave);
    argmax_merge(v, i, ov, oi);
  }
}

// Arg-max over the first `width` lanes groups (width power of two <= 64).
__device__ __forceinline__ void group_argmax(double& v, int& i, int width) {
  for (int off = width >> 1; off >= 1; off >>= 1) {
    double ov = __shfl_xor(v, off, kWave);
    int oi = __shfl_xor(i, off, kWave);
    argmax_merge(v, i, ov, oi);
  }
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, kWave));
  return v;
}

// Pivot key of a candidate row.  PARTIAL: |a| (NaN never wins).  ZERO
// (reference internal getPivot): the diagonal if non-zero, else the first
// non-zero row — encoded as 2 for a non-zero diagonal, 1 for any other
// non-zero entry, 0 for zero; ties resolve to the lowest row.
template <typename T>
__device__ __forceinline__ double pivot_key(T a, bool is_diag, int mode) {
  if (mode == 1) {
    double v = fabs((double)a);
    return v == v ? v : -1.0;
  }
  if (a == T(0)) return 0.0;
  return is_diag ? 2.0 : 1.0;
}

}  // namespace dev
}  // namespace gelim
