// GPU runtime surface of the C ABI (device selection, buffers, copies) and
// the device-side initialisers / error metric (L1/L2 on the GPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "device_common.h"
#include "gelim/internal.h"
#include "gelim/rng.h"

namespace gelim {
namespace {

__global__ __launch_bounds__(256) void copy2d_words_kernel(unsigned* __restrict__ d, int64_t dp,
                                                          const unsigned* __restrict__ sp, int64_t spp, int64_t w) {
  const unsigned* srow = sp + (int64_t)blockIdx.y * spp;
  unsigned* drow = d + (int64_t)blockIdx.y * dp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < w; i += (int64_t)gridDim.x * 256) drow[i] = srow[i];
}

// r[i] = aug[i][n] - sum_j aug[i][j] x[j] (fp64; one wave per row); with
// matvec set, r[i] = sum_j aug[i][j] x[j] (the GMRES products of the mixed
// engine).  With w, also w[i] = |b_i| + sum_j |a_ij| |x_j| in the same pass
// (the denominator of the componentwise backward error |r_i| / w_i).
__global__ __launch_bounds__(256) void residual_kernel(const double* __restrict__ aug, int64_t ld, int n,
                                                       const double* __restrict__ x, double* __restrict__ r,
                                                       int matvec, double* __restrict__ w) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const double* a = aug + (int64_t)row * ld;
  double s = 0.0, sa = 0.0;
  if (w) {
    for (int j = lane; j < n; j += 64) {
      const double av = a[j], xv = x[j];
      s = fma(av, xv, s);
      sa = fma(fabs(av), fabs(xv), sa);
    }
    sa = dev::wave_sum(sa);
  } else {
    for (int j = lane; j < n; j += 64) s = fma(a[j], x[j], s);
  }
  s = dev::wave_sum(s);
  if (lane == 0) {
    if (matvec) r[row] = s;
    else r[row] = a[n] - s;
    if (w) w[row] = sa + (matvec ? 0.0 : fabs(a[n]));
  }
}

__global__ __launch_bounds__(256) void zero_words_kernel(unsigned* __restrict__ p, int64_t nwords) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * 256) p[i] = 0u;
}

template <typename T>
__global__ void init_synthetic_kernel(T* __restrict__ A, int64_t lda, int n, int row0) {
  // A[i][j] = 2*min(i+1, j+1), b[i] = i in column n (P1i:59-69)
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = row0 + (int)blockIdx.y;
  if (j > n) return;
  T v = (j == n) ? (T)i : (T)(2 * ((j < i) ? (j + 1) : (i + 1)));
  A[(int64_t)i * lda + j] = v;
}

__global__ void init_random_kernel(double* __restrict__ A, int64_t lda, int64_t row0, int64_t col0,
                                   int ncols, uint64_t seed) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = blockIdx.y;
  if (j >= ncols) return;
  A[(int64_t)i * lda + j] = rng_uniform_pm1(seed, row0 + i, col0 + j);
}

// R[i] = sum_j A[i][j] * (j+1): one wave per row, result in column n.
template <typename T>
__global__ __launch_bounds__(256) void init_rhs_kernel(T* __restrict__ A, int64_t lda, int n) {
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (row >= n) return;
  const T* a = A + (int64_t)row * lda;
  double acc = 0.0;
  for (int j = lane; j < n; j += 64) acc += (double)a[j] * (double)(j + 1);
  acc = dev::wave_sum(acc);
  if (lane == 0) A[(int64_t)row * lda + n] = (T)acc;
}

__global__ __launch_bounds__(1024) void error_kernel(const double* __restrict__ x, int n,
                                                     double* __restrict__ out) {
  __shared__ double s[16];
  double e = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const double ref = (double)(i + 1);
    double v = fabs((x[i] - ref) / ref);
    e = (v > e || v != v) ? v : e;  // NaN propagates
  }
  // NaN-propagating max
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    double o = __shfl_xor(e, off, 64);
    e = (o > e || o != o) ? o : e;
  }
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = e;
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = 0.0;
    for (int w = 0; w < 16; ++w) m = (s[w] > m || s[w] != s[w]) ? s[w] : m;
    *out = m;
  }
}

}  // namespace

int copy2d_async(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t rows,
                 struct ihipStream_t* s) {
  if (width == 0 || rows == 0) return GELIM_OK;
  if ((width | dpitch | spitch) % 4 || ((uintptr_t)dst | (uintptr_t)src) % 4)
    return GELIM_FAIL(GELIM_E_ARG, "copy2d_async: not 4-byte aligned");
  const int64_t w = (int64_t)(width / 4);
  const unsigned bx = (unsigned)std::min<int64_t>((w + 255) / 256, 64);
  for (size_t r = 0; r < rows; r += 65535) {  // grid.y limit: one launch per 65535 rows
    const size_t nr = std::min<size_t>(65535, rows - r);
    hipLaunchKernelGGL(copy2d_words_kernel, dim3(bx, (unsigned)nr), dim3(256), 0, s,
                       static_cast<unsigned*>(dst) + r * (dpitch / 4), (int64_t)(dpitch / 4),
                       static_cast<const unsigned*>(src) + r * (spitch / 4), (int64_t)(spitch / 4), w);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

int residual_f64(const double* aug, int64_t ld, int64_t n, const double* x, double* r, hipStream_t s, int matvec,
                 double* w = nullptr) {
  hipLaunchKernelGGL(residual_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, s, aug, ld, (int)n, x, r, matvec,
                     w);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

bool coresident(int per_cu, int64_t grid) {
  if (const char* e = std::getenv("GELIM_FORCE_NONPERSISTENT"))
    if (std::atoi(e) != 0) return false;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  const int64_t usable = per_cu > 1 ? per_cu - 1 : per_cu;
  return usable * (int64_t)cus >= grid;
}

int zero_async(void* p, size_t bytes, struct ihipStream_t* s) {
  if (bytes == 0) return GELIM_OK;
  if (bytes % 4) return GELIM_FAIL(GELIM_E_ARG, "zero_async: size not a multiple of 4");
  const int64_t nw = (int64_t)(bytes / 4);
  const unsigned blocks = (unsigned)std::min<int64_t>((nw + 255) / 256, 1024);
  hipLaunchKernelGGL(zero_words_kernel, dim3(blocks), dim3(256), 0, s, static_cast<unsigned*>(p), nw);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

int init_synthetic_f64(double* A, int64_t lda, int64_t n, hipStream_t s) {
  for (int64_t r = 0; r < n; r += 65535) {  // grid.y limit
    dim3 grid((unsigned)((n + 1 + 255) / 256), (unsigned)std::min<int64_t>(65535, n - r));
    hipLaunchKernelGGL(init_synthetic_kernel<double>, grid, dim3(256), 0, s, A, lda, (int)n, (int)r);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

int init_synthetic_f32(float* A, int64_t lda, int64_t n, hipStream_t s) {
  for (int64_t r = 0; r < n; r += 65535) {  // grid.y limit
    dim3 grid((unsigned)((n + 1 + 255) / 256), (unsigned)std::min<int64_t>(65535, n - r));
    hipLaunchKernelGGL(init_synthetic_kernel<float>, grid, dim3(256), 0, s, A, lda, (int)n, (int)r);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

}  // namespace gelim

extern "C" int gelim_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int gelim_gpu_set_device(int dev) {
  HIP_TRY(hipSetDevice(dev));
  return GELIM_OK;
}

extern "C" int gelim_gpu_sync(void* stream) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return GELIM_OK;
}

extern "C" void* gelim_gpu_malloc(int64_t bytes) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, (size_t)bytes);
  if (e != hipSuccess) {
    GELIM_FAIL(GELIM_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    return nullptr;
  }
  return p;
}

extern "C" int gelim_gpu_free(void* p) {
  HIP_TRY(hipFree(p));
  return GELIM_OK;
}

extern "C" int gelim_gpu_memcpy_h2d(void* dst, const void* src, int64_t bytes, void* stream) {
  HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
  return GELIM_OK;
}

extern "C" int gelim_gpu_memcpy_d2h(void* dst, const void* src, int64_t bytes, void* stream) {
  HIP_TRY(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
  return GELIM_OK;
}

extern "C" int gelim_gpu_init_synthetic(double* dA, int64_t lda, int64_t n, void* stream) {
  if (n <= 0 || lda < n + 1) return GELIM_FAIL(GELIM_E_ARG, "init_synthetic: lda < n+1");
  return gelim::init_synthetic_f64(dA, lda, n, (hipStream_t)stream);
}

extern "C" int gelim_gpu_init_synthetic_f32(float* dA, int64_t lda, int64_t n, void* stream) {
  if (n <= 0 || lda < n + 1) return GELIM_FAIL(GELIM_E_ARG, "init_synthetic: lda < n+1");
  return gelim::init_synthetic_f32(dA, lda, n, (hipStream_t)stream);
}

extern "C" int gelim_gpu_init_random(double* dA, int64_t lda, int64_t n, uint64_t seed,
                                     void* stream) {
  if (n <= 0 || lda < n) return GELIM_FAIL(GELIM_E_ARG, "init_random: lda < n");
  return gelim_gpu_init_random_block(dA, lda, 0, n, 0, n, seed, stream);
}

extern "C" int gelim_gpu_init_random_block(double* dA, int64_t lda, int64_t row0, int64_t nrows,
                                           int64_t col0, int64_t ncols, uint64_t seed,
                                           void* stream) {
  if (nrows <= 0 || ncols <= 0) return GELIM_OK;
  if (lda < ncols) return GELIM_FAIL(GELIM_E_ARG, "init_random_block: lda < ncols");
  for (int64_t r = 0; r < nrows; r += 65535) {  // grid.y limit
    const int64_t rows = std::min<int64_t>(65535, nrows - r);
    dim3 grid((unsigned)((ncols + 255) / 256), (unsigned)rows);
    hipLaunchKernelGGL(gelim::init_random_kernel, grid, dim3(256), 0, (hipStream_t)stream,
                       dA + r * lda, lda, row0 + r, col0, (int)ncols, seed);
    HIP_TRY(hipGetLastError());
  }
  return GELIM_OK;
}

extern "C" int gelim_gpu_init_rhs(double* dA, int64_t lda, int64_t n, void* stream) {
  if (n <= 0 || lda < n + 1) return GELIM_FAIL(GELIM_E_ARG, "init_rhs: lda < n+1");
  const unsigned blocks = (unsigned)((n * 64 + 255) / 256);
  hipLaunchKernelGGL(gelim::init_rhs_kernel<double>, dim3(blocks), dim3(256), 0,
                     (hipStream_t)stream, dA, lda, (int)n);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

extern "C" int gelim_gpu_error_metric(const double* dx, int64_t n, double* d_err, void* stream) {
  hipLaunchKernelGGL(gelim::error_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, dx,
                     (int)n, d_err);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// r = b - A x for an augmented fp64 system (the refinement residual).
extern "C" int gelim_gpu_residual(const double* daug, int64_t ld, int64_t n, const double* dx, double* dr,
                                  void* stream) {
  if (n <= 0 || ld < n + 1) return GELIM_FAIL(GELIM_E_ARG, "residual: bad n / ld");
  return gelim::residual_f64(daug, ld, n, dx, dr, (hipStream_t)stream, 0);
}

// r = b - A x and w = |b| + |A| |x| in one pass (componentwise backward error).
extern "C" int gelim_gpu_residual_cw(const double* daug, int64_t ld, int64_t n, const double* dx, double* dr,
                                     double* dw, void* stream) {
  if (n <= 0 || ld < n + 1 || !dw) return GELIM_FAIL(GELIM_E_ARG, "residual_cw: bad n / ld / w");
  return gelim::residual_f64(daug, ld, n, dx, dr, (hipStream_t)stream, 0, dw);
}

// y = A x for the n x n matrix of an augmented fp64 system.
extern "C" int gelim_gpu_matvec(const double* daug, int64_t ld, int64_t n, const double* dx, double* dy, void* stream) {
  if (n <= 0 || ld < n) return GELIM_FAIL(GELIM_E_ARG, "matvec: bad n / ld");
  return gelim::residual_f64(daug, ld, n, dx, dy, (hipStream_t)stream, 1);
}
