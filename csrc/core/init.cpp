// L1/L2 initialisers and the error metric (host side).
//
//  synthetic : A[i][j] = 2*min(i+1, j+1), b[i] = i
//              (Pthreads/Version-1/gauss_internal_input.c:59-69). SPD, exact
//              solution (-0.5, 0, ..., 0, 0.5).
//  random    : U[-1,1) from a counter-based hash so host and device produce
//              bit-identical matrices (used by the benchmark: "synthetic
//              random-init matrices", BASELINE.json north_star).
//  rhs       : R = A * (1..n)   (gauss_external_input.c:90-108)
//  error     : max_i |x_i - X__i| / |X__i|   (gauss_external_input.c:308-315)
#include <cmath>
#include <cstdint>

#include "gelim/internal.h"
#include "gelim/rng.h"

extern "C" void gelim_init_synthetic_f64(double* A, int64_t lda, double* b,
                                         int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    double* row = A + i * lda;
    for (int64_t j = 0; j < n; ++j) row[j] = (j < i) ? 2.0 * (j + 1) : 2.0 * (i + 1);
    if (b) b[i] = (double)i;
  }
}

extern "C" void gelim_init_random_f64(double* A, int64_t lda, int64_t n,
                                      uint64_t seed) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) A[i * lda + j] = gelim::rng_uniform_pm1(seed, i, j);
}

extern "C" void gelim_init_random_block_f64(double* out, int64_t ld, int64_t row0,
                                            int64_t nrows, int64_t col0, int64_t ncols,
                                            uint64_t seed) {
  for (int64_t r = 0; r < nrows; ++r)
    for (int64_t c = 0; c < ncols; ++c)
      out[r * ld + c] = gelim::rng_uniform_pm1(seed, row0 + r, col0 + c);
}

extern "C" void gelim_init_rhs_f64(const double* A, int64_t lda, double* R,
                                   int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    double acc = 0.0;
    const double* row = A + i * lda;
    for (int64_t j = 0; j < n; ++j) acc += row[j] * (double)(j + 1);
    R[i] = acc;
  }
}

extern "C" double gelim_error_metric(const double* x, int64_t n) {
  double err = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    double ref = (double)(i + 1);
    double e = std::fabs((x[i] - ref) / ref);
    if (e > err || std::isnan(e)) err = std::isnan(e) ? NAN : e;
    if (std::isnan(err)) break;
  }
  return err;
}

extern "C" void gelim_init_matmul_f32(float* A, float* B, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < n; ++j) {
      int64_t idx = j + i * n;
      A[idx] = (float)idx + 1.0f;
      B[idx] = 1.0f / ((float)idx + 1.0f);
    }
}
