// CPU fp32 matmul baselines: the exact reference i-j-k loops that serve as the
// speedup denominator (CUDA_and_OpenMP/Version-2/cuda_matmul.cu:28-57).
// The sequential loop is deliberately left naive (column walk of B): the
// benchmark must divide by the SAME loop the reference used.
#include <cstdint>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "gelim/internal.h"

namespace {

__attribute__((noinline)) void matmul_rows(const float* A, const float* B,
                                           float* C, int64_t n, int64_t i) {
  for (int64_t j = 0; j < n; j++) {
    float temp = 0.0f;
    for (int64_t k = 0; k < n; k++) temp += A[k + i * n] * B[j + k * n];
    C[j + i * n] = temp;
  }
}

}  // namespace

extern "C" void gelim_cpu_matmul_f32(const float* A, const float* B, float* C,
                                     int64_t n, int omp, int threads) {
  if (!omp) {
    for (int64_t i = 0; i < n; i++) matmul_rows(A, B, C, n, i);
    return;
  }
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#endif
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; i++) matmul_rows(A, B, C, n, i);
}
