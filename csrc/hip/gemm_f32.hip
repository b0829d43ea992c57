// fp32 matrix multiply C = A * B on MI355X (row-major, C is M x N).
//
//  NAIVE_ROW  (K1 parity, CUDA_and_OpenMP/Version-1/cuda_matmul.cu:89-103):
//             one workgroup per output row, threads stride the columns.
//  NAIVE_ELEM (K2 parity, CUDA_and_OpenMP/Version-2/cuda_matmul.cu:89-101):
//             2-D grid, one thread per output element.
//  MFMA       (K3', absent in the reference): LDS-tiled GEMM on the exact-fp32
//             matrix cores (v_mfma_f32_32x32x2_f32), LDS double-buffered with
//             one barrier per K-step, XCD-aware tile order.  4 wave64s per
//             workgroup in a 2x2 arrangement; 64x64x16 tiles (one 32x32 MFMA
//             block per wave, four workgroups per CU) or, when there are at
//             least 2 128x128 tiles per CU, 128x64x16 tiles (2x1 blocks per
//             wave).  LDS holds A transposed ([k][m]) and B as is ([k][n]), so
//             both fragment reads are unit-stride across lanes; A rows padded
//             by 2 floats, B rows by 4: no LDS bank conflicts (SQ_LDS_BANK_
//             CONFLICT = 0; 14 % of the LDS cycles with A padded by 4,
//             profiles/gemm_microbench.txt).
// The naive kernels use 64-bit indexing (the reference's int products
// overflow for n > 46340).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

struct Mat {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int M, N, K, acc;
  float alpha;  // MFMA path: C (+)= alpha * A B (the blocked no-pivot LU's update passes -1)
  double* C64 = nullptr;  // MFMA path: an fp64 C instead (fp32 products, fp64 accumulation in C)
};

__global__ void naive_row_kernel(Mat p) {
  const int64_t i = blockIdx.x;
  for (int64_t j = threadIdx.x; j < p.N; j += blockDim.x) {
    float temp = 0.0f;
    for (int64_t k = 0; k < p.K; ++k) temp += p.A[i * p.lda + k] * p.B[k * p.ldb + j];
    float* c = p.C + i * p.ldc + j;
    *c = p.acc ? *c + temp : temp;
  }
}

__global__ void naive_elem_kernel(Mat p) {
  const int64_t j = threadIdx.x + (int64_t)blockIdx.y * blockDim.x;
  const int64_t i = blockIdx.x;
  if (j >= p.N) return;
  float temp = 0.0f;
  for (int64_t k = 0, kn = 0; k < p.K; ++k, kn += p.ldb) temp += p.A[i * p.lda + k] * p.B[j + kn];
  float* c = p.C + i * p.ldc + j;
  *c = p.acc ? *c + temp : temp;
}

// Two tile shapes, picked per problem by the number of tiles per CU:
//  * 64 x 64 x 16 when 128 x 128 tiles would leave fewer than 2 per CU (2048^2:
//    1024 workgroups, four co-resident per CU, so one workgroup's LDS store +
//    barrier hides under the others' MFMAs: 128x128 179 us, 128x64 170 us,
//    64x64 166 us at 2048^2);
//  * 128 x 64 x 16 (each wave 64 x 32 = 2 x 1 MFMA blocks) for larger
//    problems (>= 2 128x128 tiles per CU): 125 TF at 8192^2, 124 at 16384^2
//    vs 120-121 for 128 x 128 x 32 (GELIM_SGEMM_SHAPE picks any compiled
//    shape for A/B runs).
constexpr int kMmThreads = 256;
// APAD = 2: a row stride = 2 mod 8 floats puts the 4 k-chunks of the transposed A
// stores on distinct bank octets (APAD = 4: 2-way, 14 % of the LDS cycles)
constexpr int APAD = 2, BPAD = 4;

template <int BM, int BN, int BK>
struct Tile {
  static constexpr int WM = BM / 2, WN = BN / 2;  // rows / columns per wave (2 x 2 waves)
  // float4s per thread for one A (BM x BK, k fastest) / B (BK x BN) tile
  static constexpr int kFA = BM * BK / 4 / kMmThreads, kFB = BK * BN / 4 / kMmThreads;
  static_assert(kFA * 4 * kMmThreads == BM * BK && kFB * 4 * kMmThreads == BK * BN, "tile / threads");
  struct Frag {
    float4 a[kFA];  // A tile: row = idx / (BK/4), k = 4 (idx % (BK/4)), idx = t + 256 h
    float4 b[kFB];  // B tile: k = idx / (BN/4), col = 4 (idx % (BN/4))
  };
};

template <bool CHECK, int BM, int BN, int BK>
__device__ __forceinline__ void load_tiles(typename Tile<BM, BN, BK>::Frag& f, const Mat& p, int m0, int n0,
                                           int k0) {
  constexpr int kFA = Tile<BM, BN, BK>::kFA, kFB = Tile<BM, BN, BK>::kFB;
  const float* __restrict__ A = p.A;
  const float* __restrict__ B = p.B;
  const int M = p.M, N = p.N, K = p.K;
  const int64_t lda = p.lda, ldb = p.ldb;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < kFA; ++h) {
    const int idx = t + kMmThreads * h;
    const int row = idx / (BK / 4), kc = (idx % (BK / 4)) * 4;
    const int gm = m0 + row, gk = k0 + kc;
    if (!CHECK) {
      f.a[h] = *reinterpret_cast<const float4*>(A + (int64_t)gm * lda + gk);
    } else {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (gm < M && gk + e < K) ? A[(int64_t)gm * lda + gk + e] : 0.f;
      f.a[h] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
#pragma unroll
  for (int h = 0; h < kFB; ++h) {
    const int idx = t + kMmThreads * h;
    const int kr = idx / (BN / 4), nc = (idx % (BN / 4)) * 4;
    const int gkb = k0 + kr, gn = n0 + nc;
    if (!CHECK) {
      f.b[h] = *reinterpret_cast<const float4*>(B + (int64_t)gkb * ldb + gn);
    } else {
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (gkb < K && gn + e < N) ? B[(int64_t)gkb * ldb + gn + e] : 0.f;
      f.b[h] = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
}

template <int BM, int BN, int BK>
__device__ __forceinline__ void store_tiles(const typename Tile<BM, BN, BK>::Frag& f, float (*As)[BM + APAD],
                                            float (*Bs)[BN + BPAD]) {
  constexpr int kFA = Tile<BM, BN, BK>::kFA, kFB = Tile<BM, BN, BK>::kFB;
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < kFA; ++h) {
    const int idx = t + kMmThreads * h;
    const int row = idx / (BK / 4), kc = (idx % (BK / 4)) * 4;
    As[kc + 0][row] = f.a[h].x;
    As[kc + 1][row] = f.a[h].y;
    As[kc + 2][row] = f.a[h].z;
    As[kc + 3][row] = f.a[h].w;
  }
#pragma unroll
  for (int h = 0; h < kFB; ++h) {
    const int idx = t + kMmThreads * h;
    const int kr = idx / (BN / 4), nc = (idx % (BN / 4)) * 4;
    *reinterpret_cast<float4*>(&Bs[kr][nc]) = f.b[h];
  }
}

template <bool CHECK, int BM, int BN, int BK>
__global__ __launch_bounds__(kMmThreads, 2) void mfma_gemm_kernel(Mat p, int tiles_n, int ntiles) {
  using TL = Tile<BM, BN, BK>;
  constexpr int WM = TL::WM, WN = TL::WN;
  const int M = p.M, N = p.N, K = p.K;
  __shared__ __attribute__((aligned(16))) float As[2][BK][BM + APAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][BK][BN + BPAD];

  // XCD-aware bijective remap: consecutive tiles (sharing A row panels) go to
  // the same XCD's L2 (cdna_hip_programming.md §5.5 T1).
  const int orig = blockIdx.x;
  const int q = ntiles / 8, rem = ntiles % 8, xcd = orig % 8;
  const int tile = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + orig / 8;
  const int m0 = (tile / tiles_n) * BM, n0 = (tile % tiles_n) * BN;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = (wave >> 1) * WM, wn = (wave & 1) * WN;
  const int l31 = lane & 31, kh = lane >> 5;

  constexpr int MI = WM / 32, NJ = WN / 32;
  dev::f16x acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // LDS double buffer + TWO register fragments in flight: tile kt+1 is stored
  // to LDS during step kt from registers loaded two steps earlier, so a
  // global load has two K-steps of MFMA work (not one) to land under
  const int nk = (K + BK - 1) / BK;
  typename TL::Frag fa, fb;
  load_tiles<CHECK, BM, BN, BK>(fa, p, m0, n0, 0);
  store_tiles<BM, BN, BK>(fa, As[0], Bs[0]);
  if (nk > 1) load_tiles<CHECK, BM, BN, BK>(fa, p, m0, n0, BK);
  if (nk > 2) load_tiles<CHECK, BM, BN, BK>(fb, p, m0, n0, 2 * BK);
  __syncthreads();

  // one K-step: MFMAs on LDS buffer kt&1; fnext (tile kt+1) goes to the other
  // buffer and its registers are reloaded with tile kt+3
  auto kstep = [&](int kt, typename TL::Frag& fnext) {
    const int cur = kt & 1;
#pragma unroll
    for (int k = 0; k < BK; k += 2) {
      const int kk = k + kh;
      float ai[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) ai[i] = As[cur][kk][wm + 32 * i + l31];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float bj = Bs[cur][kk][wn + 32 * j + l31];
#pragma unroll
        for (int i = 0; i < MI; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ai[i], bj, acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) store_tiles<BM, BN, BK>(fnext, As[cur ^ 1], Bs[cur ^ 1]);
    if (kt + 3 < nk) load_tiles<CHECK, BM, BN, BK>(fnext, p, m0, n0, (kt + 3) * BK);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    kstep(kt, fa);
    if (kt + 1 < nk) kstep(kt + 1, fb);
  }

  // epilogue: C/D map of 32x32 f32 MFMA: col = l&31, row = (r&3) + 8(r>>2) + 4(l>>5)
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = n0 + wn + 32 * j + l31;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * kh;
        if (!CHECK || (row < M && col < N)) {
          const float v = p.alpha * acc[i][j][r];
          if (p.C64) {
            double* c = p.C64 + (int64_t)row * p.ldc + col;
            *c = p.acc ? *c + (double)v : (double)v;
          } else {
            float* c = p.C + (int64_t)row * p.ldc + col;
            *c = p.acc ? *c + v : v;
          }
        }
      }
    }
}

template <int M_, int N_, int K_>
struct Shape {
  static constexpr int BM = M_, BN = N_, BK = K_;
};

}  // namespace

int matmul_f32(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
               int64_t M, int64_t N, int64_t K, int accumulate, int kernel, hipStream_t s, float alpha,
               double* C64 = nullptr) {
  if (M <= 0 || N <= 0 || K <= 0) return GELIM_FAIL(GELIM_E_ARG, "matmul: bad shape");
  if (alpha != 1.0f && kernel != GELIM_MM_MFMA) return GELIM_FAIL(GELIM_E_ARG, "matmul: alpha needs the MFMA kernel");
  if (M > INT32_MAX || N > INT32_MAX || K > INT32_MAX)
    return GELIM_FAIL(GELIM_E_ARG, "matmul: dimension exceeds 2^31");
  if (lda < K || ldb < N || ldc < N) return GELIM_FAIL(GELIM_E_ARG, "matmul: leading dimension too small");
  if (C64 && kernel != GELIM_MM_MFMA) return GELIM_FAIL(GELIM_E_ARG, "matmul: an fp64 C needs the MFMA kernel");
  Mat p{A, lda, B, ldb, C, ldc, (int)M, (int)N, (int)K, accumulate, alpha, C64};
  switch (kernel) {
    case GELIM_MM_NAIVE_ROW: {
      const int threads = (int)std::min<int64_t>(1024, N);
      hipLaunchKernelGGL(naive_row_kernel, dim3((unsigned)M), dim3(threads), 0, s, p);
      break;
    }
    case GELIM_MM_NAIVE_ELEM: {
      const int threads = (int)std::min<int64_t>(1024, N);
      dim3 grid((unsigned)M, (unsigned)((N + 1023) / 1024));
      hipLaunchKernelGGL(naive_elem_kernel, grid, dim3(threads), 0, s, p);
      break;
    }
    case GELIM_MM_MFMA: {
      int cus = 256, dev = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const int64_t big_tiles = ((M + 127) / 128) * ((N + 127) / 128);
      const bool big = big_tiles >= 2 * (int64_t)cus;
      auto launch = [&](auto tag) {
        constexpr int BM = decltype(tag)::BM, BN = decltype(tag)::BN, BK = decltype(tag)::BK;
        const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
        const int ntiles = tiles_m * tiles_n;
        const bool aligned = (M % BM == 0) && (N % BN == 0) && (K % BK == 0) && (lda % 4 == 0) &&
                             (ldb % 4 == 0) && ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0);
        if (aligned)
          hipLaunchKernelGGL((mfma_gemm_kernel<false, BM, BN, BK>), dim3(ntiles), dim3(kMmThreads), 0, s, p,
                             tiles_n, ntiles);
        else
          hipLaunchKernelGGL((mfma_gemm_kernel<true, BM, BN, BK>), dim3(ntiles), dim3(kMmThreads), 0, s, p,
                             tiles_n, ntiles);
      };
      // measured (profiles/gemm_microbench.txt, round 2): 128x64x16 is the
      // fastest shape once there are >= 2 128x128 tiles per CU (8192^2: 125
      // vs 120 TF for 128x128x32), 64x64x16 below (2048^2); 64x64x32,
      // 128x128x32, 128x64x32 and 64x128x16 were slower at both
      if (big) launch(Shape<128, 64, 16>{});
      else launch(Shape<64, 64, 16>{});
      break;
    }
    default:
      return GELIM_FAIL(GELIM_E_ARG, "matmul: unknown kernel");
  }
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace gelim

extern "C" int gelim_gpu_matmul_f32(const float* dA, const float* dB, float* dC, int64_t M,
                                    int64_t N, int64_t K, int kernel, void* stream) {
  return gelim::matmul_f32(dA, K, dB, N, dC, N, M, N, K, 0, kernel, (hipStream_t)stream, 1.0f);
}

extern "C" int gelim_gpu_matmul_f32_ex(const float* dA, int64_t lda, const float* dB, int64_t ldb,
                                       float* dC, int64_t ldc, int64_t M, int64_t N, int64_t K,
                                       int accumulate, int kernel, void* stream) {
  return gelim::matmul_f32(dA, lda, dB, ldb, dC, ldc, M, N, K, accumulate, kernel,
                           (hipStream_t)stream, 1.0f);
}
