// GPU runtime surface of the C ABI (device selection, buffers, copies) and
// the device-side initialisers / error metric (L1/L2 on the GPU).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "device_common.h"
#include "gelim/internal.h"
#include "gelim/rng.h"

namespace gelim {
namespace {

// (Write-through stores here measured within noise of plain ones, round 4,
// profiles/dgemm_wt_r4.txt.)
__global__ __launch_bounds__(256) void copy2d_words_kernel(unsigned* __restrict__ d, int64_t dp,
                                                          const unsigned* __restrict__ sp, int64_t spp, int64_t w) {
  const unsigned* srow = sp + (int64_t)blockIdx.y * spp;
  unsigned* drow = d + (int64_t)blockIdx.y * dp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < w; i += (int64_t)gridDim.x * 256) drow[i] = srow[i];
}

// 8-byte elements (fp64 rows: the solvers' input staging), four per thread in
// flight, coalesced; rows grid-strided so a large copy is a few thousand
// workgroups, not one per (row, 1024 columns): 8192 x 8193 was dispatch-bound
// at 2.4 TB/s with 74k workgroups
constexpr int kCopyPer = 4;
constexpr int kCopyRowsGrid = 1024;
__global__ __launch_bounds__(256) void copy2d_u64_kernel(uint64_t* __restrict__ d, int64_t dp,
                                                         const uint64_t* __restrict__ sp, int64_t spp, int64_t w,
                                                         int64_t rows) {
  const int64_t base = (int64_t)blockIdx.x * 256 * kCopyPer + threadIdx.x;
  for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) {
    const uint64_t* srow = sp + r * spp;
    uint64_t* drow = d + r * dp;
    uint64_t v[kCopyPer];
#pragma unroll
    for (int k = 0; k < kCopyPer; ++k) {
      const int64_t i = base + 256 * k;
      v[k] = i < w ? srow[i] : 0;
    }
#pragma unroll
    for (int k = 0; k < kCopyPer; ++k) {
      const int64_t i = base + 256 * k;
      if (i < w) drow[i] = v[k];
    }
  }
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

struct FillSet {
  unsigned* p[kMaxFills];
  int64_t nw[kMaxFills];
  unsigned v[kMaxFills];
  int nf;
};

__global__ __launch_bounds__(256) void fill_words_kernel(FillSet fs) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int f = 0; f < fs.nf; ++f)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < fs.nw[f]; i += stride) fs.p[f][i] = fs.v[f];
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
  const bool u64 = (width | dpitch | spitch) % 8 == 0 && ((uintptr_t)dst | (uintptr_t)src) % 8 == 0;
  if (u64) {
    const int64_t w = (int64_t)(width / 8);
    const unsigned bx = (unsigned)((w + 256 * kCopyPer - 1) / (256 * kCopyPer));
    const unsigned by = (unsigned)std::min<size_t>(rows, kCopyRowsGrid);
    hipLaunchKernelGGL(copy2d_u64_kernel, dim3(bx, by), dim3(256), 0, s, static_cast<uint64_t*>(dst),
                       (int64_t)(dpitch / 8), static_cast<const uint64_t*>(src), (int64_t)(spitch / 8), w,
                       (int64_t)rows);
    HIP_TRY(hipGetLastError());
    return GELIM_OK;
  }
  for (size_t r = 0; r < rows; r += 65535) {  // grid.y limit: one launch per 65535 rows
    const size_t nr = std::min<size_t>(65535, rows - r);
    {
      const int64_t w = (int64_t)(width / 4);
      const unsigned bx = (unsigned)std::min<int64_t>((w + 255) / 256, 64);
      hipLaunchKernelGGL(copy2d_words_kernel, dim3(bx, (unsigned)nr), dim3(256), 0, s,
                         static_cast<unsigned*>(dst) + r * (dpitch / 4), (int64_t)(dpitch / 4),
                         static_cast<const unsigned*>(src) + r * (spitch / 4), (int64_t)(spitch / 4), w);
    }
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

int fill_words_async(const WordFill* f, int nf, struct ihipStream_t* s) {
  if (nf < 0 || nf > kMaxFills) return GELIM_FAIL(GELIM_E_ARG, "fill_words_async: too many ranges");
  FillSet fs{};
  int64_t most = 0;
  for (int k = 0; k < nf; ++k) {
    if (f[k].bytes % 4 || (uintptr_t)f[k].p % 4) return GELIM_FAIL(GELIM_E_ARG, "fill_words_async: not 4-byte aligned");
    fs.p[fs.nf] = static_cast<unsigned*>(f[k].p);
    fs.nw[fs.nf] = (int64_t)(f[k].bytes / 4);
    fs.v[fs.nf] = f[k].value;
    most = std::max(most, fs.nw[fs.nf]);
    fs.nf += f[k].bytes ? 1 : 0;
  }
  if (!fs.nf) return GELIM_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((most + 255) / 256, 1024);
  hipLaunchKernelGGL(fill_words_kernel, dim3(blocks), dim3(256), 0, s, fs);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
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

// ---- side streams on a hardware queue of their own ---------------------------
// HIP maps streams onto at most GPU_MAX_HW_QUEUES hardware queues per process
// and shares queues once they run out.  A lookahead side stream that shares
// the caller's queue runs AFTER the caller's work instead of beside it: the
// 8192 solve took 49.4 instead of 33.9 ms, the distributed 2048 solve 16 instead
// of 8 ms, depending on how many streams the process had created before
// (profiles/hw_queues_r4.txt).  So a side stream is probed when it is made:
// a kernel on the default stream waits (bounded, 5 ms) for a flag that a
// kernel on the new stream sets -- it sees the flag only if the two run
// concurrently.  A stream that failed is parked (kept alive, so the runtime
// does not hand its queue out again) and another one is made, up to 8 times.
namespace {
constexpr unsigned long long kProbeTicks = 500000ull;  // 5 ms at 100 MHz

__global__ void probe_wait_kernel(int* w, unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  int seen = 0;
  for (;;) {
    if (__hip_atomic_load(&w[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      seen = 1;
      break;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) break;
    __builtin_amdgcn_s_sleep(2);
  }
  __hip_atomic_store(&w[1], seen ? 1 : 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void probe_set_kernel(int* w) {
  if (threadIdx.x == 0) __hip_atomic_store(&w[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

std::mutex g_park_mu;
// Streams that shared a queue with the stream they were probed against.  They
// stay alive while parked (so the runtime does not hand their queue out
// again during the same search) and are offered first to the next search;
// the pool is capped, past the cap a failed stream is destroyed.
constexpr size_t kParkCap = 12;
std::vector<hipStream_t> g_parked;
int g_side_stats[2] = {0, 0};  // {probed streams, streams found sharing a queue} (diagnostics)

// 1: `setter` runs concurrently with `waiter`, 0: it does not (they share a
// hardware queue), < 0: error
int probe_pair(hipStream_t waiter, hipStream_t setter, int* w) {
  int h[2] = {0, 0};
  HIP_TRY(hipMemsetAsync(w, 0, 2 * sizeof(int), waiter));
  HIP_TRY(hipStreamSynchronize(waiter));
  hipLaunchKernelGGL(probe_wait_kernel, dim3(1), dim3(64), 0, waiter, w, kProbeTicks);
  hipLaunchKernelGGL(probe_set_kernel, dim3(1), dim3(64), 0, setter, w);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(setter));
  HIP_TRY(hipStreamSynchronize(waiter));
  HIP_TRY(hipMemcpy(h, w, sizeof(h), hipMemcpyDeviceToHost));
  return h[1] == 1 ? 1 : 0;
}

// 1 when s runs beside the default stream AND beside every stream of
// others[0..nothers), 0 when it shares a queue with one of them
int probe_all(hipStream_t s, hipStream_t const* others, int nothers, int* w) {
  int ok = probe_pair(nullptr, s, w);
  for (int i = 0; ok == 1 && i < nothers; ++i)
    if (others[i]) ok = probe_pair(others[i], s, w);
  return ok;
}

void park(hipStream_t s) {
  if (g_parked.size() < kParkCap) {
    g_parked.push_back(s);
  } else {
    (void)hipStreamDestroy(s);
  }
}
}  // namespace

bool probe_enabled() {
  const char* e = std::getenv("GELIM_SIDE_PROBE");  // 0: plain streams, no probe
  return !(e && std::atoi(e) == 0);
}

// one probe word pair per device for the process (no hipFree: it would
// synchronise the whole device under other threads' work); call under g_park_mu
int probe_words(int** w) {
  static int* words[64] = {};
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return GELIM_FAIL(GELIM_E_ARG, "side stream: device index");
  if (!words[dev]) HIP_TRY(hipMalloc((void**)&words[dev], 2 * sizeof(int)));
  *w = words[dev];
  return GELIM_OK;
}

// A stream concurrent with the default stream and with others[0..nothers):
// parked streams of earlier searches are tried first, then up to 8 new ones.
// (Stream priorities for the side streams and for hip-rbt's chain were
// measured without gain in round 4, profiles/stream_prio_r4.txt.)
int probed_stream_create(hipStream_t* out, hipStream_t const* others, int nothers) {
  *out = nullptr;
  if (!probe_enabled()) {
    HIP_TRY(hipStreamCreateWithFlags(out, hipStreamNonBlocking));
    return GELIM_OK;
  }
  std::lock_guard<std::mutex> lk(g_park_mu);  // one probe at a time (shared words)
  int* w = nullptr;
  GELIM_TRY(probe_words(&w));
  {
    for (size_t i = 0; i < g_parked.size(); ++i) {
      const int ok = probe_all(g_parked[i], others, nothers, w);
      ++g_side_stats[0];
      if (ok < 0) return ok;
      if (ok == 1) {
        *out = g_parked[i];
        g_parked.erase(g_parked.begin() + (ptrdiff_t)i);
        return GELIM_OK;
      }
      ++g_side_stats[1];
    }
  }
  hipStream_t s = nullptr;
  int rc = GELIM_OK;
  for (int attempt = 0; attempt < 8; ++attempt) {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      rc = GELIM_FAIL(GELIM_E_HIP, "side stream");
      s = nullptr;
      break;
    }
    const int ok = probe_all(s, others, nothers, w);
    ++g_side_stats[0];
    if (ok != 0 || attempt == 7) break;  // concurrent, an error (keep the stream), or out of tries
    ++g_side_stats[1];
    park(s);
    s = nullptr;
  }
  *out = s;
  return s ? GELIM_OK : rc;
}

int side_stream_create(hipStream_t* out) { return probed_stream_create(out, nullptr, 0); }

}  // namespace gelim

// A non-blocking stream that runs concurrently with the default stream
// (probed; see side_stream_create).  Destroy with gelim_gpu_stream_destroy.
extern "C" int gelim_gpu_side_stream_create(void** out) {
  hipStream_t s = nullptr;
  GELIM_TRY(gelim::side_stream_create(&s));
  *out = (void*)s;
  return GELIM_OK;
}

// {least, greatest} stream priority of the current device
extern "C" int gelim_gpu_stream_priority_range(int32_t* out) {
  int least = 0, greatest = 0;
  HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
  out[0] = least;
  out[1] = greatest;
  return GELIM_OK;
}

extern "C" int gelim_gpu_stream_destroy(void* s) {
  if (s) HIP_TRY(hipStreamDestroy((hipStream_t)s));
  return GELIM_OK;
}

// 1 when `stream` (an existing stream, e.g. one of torch's pool) runs
// concurrently with the default stream, 0 when it shares its hardware queue
// (always 1 with GELIM_SIDE_PROBE=0), < 0 on errors.
extern "C" int gelim_gpu_stream_probe(void* stream) {
  if (!gelim::probe_enabled()) return 1;
  std::lock_guard<std::mutex> lk(gelim::g_park_mu);
  int* w = nullptr;
  GELIM_TRY(gelim::probe_words(&w));
  const int ok = gelim::probe_pair(nullptr, (hipStream_t)stream, w);
  if (ok >= 0) {
    ++gelim::g_side_stats[0];
    if (ok == 0) ++gelim::g_side_stats[1];
  }
  return ok;
}

// A new non-blocking stream that runs concurrently with the default stream
// and with each of others[0..nothers) (null entries skipped): the streams a
// rank keeps busy at once -- main, the lookahead side stream and the stream
// its collectives run on -- each on a hardware queue of its own.
extern "C" int gelim_gpu_stream_create_probed(void** out, void* const* others, int32_t nothers) {
  if (nothers < 0 || nothers > 16) return GELIM_FAIL(GELIM_E_ARG, "stream_create_probed: nothers");
  hipStream_t s = nullptr;
  GELIM_TRY(gelim::probed_stream_create(&s, (hipStream_t const*)others, nothers));
  *out = (void*)s;
  return GELIM_OK;
}

// One half of a concurrency probe on caller-chosen streams and words (two
// ints, zeroed by the caller): role 0 launches the bounded waiter (words[1]
// becomes 1 if it saw words[0] set within `ticks` 100 MHz ticks, else 2),
// role 1 the setter.  Used to check that a collective queued on one stream
// does not serialise behind a kernel on another (parallel/comm.py).
extern "C" int gelim_gpu_probe_kernel(void* stream, int32_t* words, int32_t role, int64_t ticks) {
  if (role == 0) {
    hipLaunchKernelGGL(gelim::probe_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, words,
                       (unsigned long long)std::max<int64_t>(1, ticks));
  } else {
    hipLaunchKernelGGL(gelim::probe_set_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, words);
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

// {streams probed, streams that shared the default stream's queue}
extern "C" void gelim_gpu_side_stream_stats(int32_t* out) {
  std::lock_guard<std::mutex> lk(gelim::g_park_mu);
  out[0] = gelim::g_side_stats[0];
  out[1] = gelim::g_side_stats[1];
}

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
