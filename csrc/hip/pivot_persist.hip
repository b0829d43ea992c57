// The reference's per-pivot Gaussian elimination as ONE persistent launch
// (GaussSolver backend "hip-pivot", n <= 2048 on one MI355X).
//
// The reference runs one pivot search + one elimination sweep per column,
// with a fork/join (Pthreads V1/V2, OpenMP) or a condvar barrier (Pthreads
// V3, thread 0 alone doing getPivot while the others wait) between them
// (Pthreads/Version-3/gauss_internal_input.c:150-202,
// OpenMP_and_MPI/gauss_openmp/gauss_external_input.c:153-182).  The two-kernel
// form (gauss_pivot.hip) pays two dependent launches per column (~12 us a
// step at 2048).  Here the whole elimination is one grid of G workgroups, one
// per CU, all co-resident, and the matrix lives in REGISTERS for the whole
// factorisation:
//  * workgroup w owns the physical rows w, w + G, ... (R rows); thread t
//    owns the columns t, t + NT, ... (KC slots) of each of them, so every
//    element of the 2048 x 2049 system has one home VGPR on the chip and is
//    never re-read from memory until the final write-back;
//  * rows never move (logical pivoting): every workgroup keeps the position
//    -> row map in LDS and its rows' positions in registers; the final
//    write-back stores each row at its position, which is the LAPACK-style
//    result of the two-kernel form (full-width swaps, multipliers in place,
//    ipiv / diag), so back substitution and resolve() are shared;
//  * per column i, TWO one-hop exchanges and one workgroup barrier:
//      candidate: the thread owning column i of each workgroup (it updated
//        that column first, at the end of step i-1) publishes its rows' best
//        (key, position) as one data-tagged 16-byte granule; wave 0 of every
//        workgroup sweeps all G granules (4 per lane) and finds the pivot --
//        the same choice in every workgroup;
//      pivot row: the owner of the pivot row scales it (true division, as the
//        reference) and every thread publishes its columns of it as tagged
//        granules; every thread of every workgroup polls only the granules of
//        ITS columns, then updates them in its rows -- no flag, no drain,
//        no second barrier;
//    tags are the step number, buffers are parity double-buffered (a slot is
//    rewritten two steps later, after every workgroup has provably read it);
//  * every spin is bounded (200 ms of s_memrealtime) and reports through the
//    plan's error word, which every spinner also polls, so the grid drains.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>

#include "device_common.h"
#include "gelim/internal.h"

namespace gelim {
namespace {

constexpr unsigned long long kSpinTicks = 20000000ull;  // 200 ms at 100 MHz
constexpr int kAuxSc1 = 16;                             // buffer-op aux: sc1 (write-through store, L1-bypass load)
constexpr int kPpErr = 9;                               // info[1] code: a pivot hand-off timed out

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long rtc() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void put16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint64_t a, unsigned b, unsigned c) {
  const u32x4 v = {(unsigned)a, (unsigned)(a >> 32), b, c};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, kAuxSc1);
}

__device__ __forceinline__ u32x4 get16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, kAuxSc1);
}

// Order-preserving key of a candidate (0 = no candidate; a live row always
// has a key >= 1, and a best key <= 1 means the column is zero -- singular).
// PARTIAL: bits(|a|) + 1 (NaN ranks as zero); ZERO (the internal programs'
// rule): 3 non-zero at the diagonal position, 2 other non-zero, 1 zero.
template <typename T>
__device__ __forceinline__ uint64_t cand_key(T a, bool diag, int mode) {
  const double v = (double)a;
  if (mode == 1) {
    const uint64_t bits = (uint64_t)__double_as_longlong(v) & 0x7fffffffffffffffull;
    return bits > 0x7ff0000000000000ull ? 1 : bits + 1;
  }
  return v == 0.0 ? 1 : (diag ? 3 : 2);
}

struct PpArgs {
  void* A;          // n x (n+1) augmented system (row-major, lda), factored in place
  int64_t lda;
  int n, mode;
  int* info;        // [0] 1 + first zero-pivot column, [1] error word
  int* ipiv;        // [n] LAPACK interchange: position of the pivot row at step i
  double* diag;     // [n] pivot values
  unsigned char* cand;  // [2][G] 16-byte candidate granules
  unsigned char* rowb;  // [2][n+1] 16-byte pivot-row granules
};

// out[r] = a[r][kc] for a thread-uniform kc, by a branch to the one
// compile-time slot (a select chain costs R x KC x 2 v_cndmask)
template <int K, int KC, typename T, int R>
__device__ __forceinline__ void column_of_k(const T (&a)[R][KC], int kc, T (&out)[R]) {
  if constexpr (K < KC) {
    if (kc == K) {
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = a[r][K];
    } else {
      column_of_k<K + 1, KC>(a, kc, out);
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = T(0);
  }
}
template <int KC, typename T, int R>
__device__ __forceinline__ void column_of(const T (&a)[R][KC], int kc, T (&out)[R]) {
  column_of_k<0, KC>(a, kc, out);
}

template <typename T, int NT, int R, int KC>
__global__ __launch_bounds__(NT) void pivot_persist_kernel(PpArgs g) {
  extern __shared__ int rowat[];  // [n] position -> physical row; then scalars
  const int n = g.n, G = (int)gridDim.x, w = (int)blockIdx.x;
  const int t = (int)threadIdx.x, lane = t & 63, wave = t >> 6;
  int* s_ctl = rowat + n;                              // [0] p, [1] ppos, [2] singular, [3] abort
  T* s_m = reinterpret_cast<T*>(rowat + ((n + 8 + 3) & ~3));  // [2][R] column-i values (the multipliers), 16-byte aligned
  T* s_best = s_m + 2 * R;                             // [2] this workgroup's candidate value
  T* A = static_cast<T*>(g.A);
  const __amdgpu_buffer_rsrc_t crs = rsrc(g.cand, (uint32_t)(2 * G * 16));
  const __amdgpu_buffer_rsrc_t rrs = rsrc(g.rowb, (uint32_t)(2 * (n + 1) * 16));
  int* err = g.info + 1;

  // ---- registers: R rows x KC column slots ------------------------------------
  T a[R][KC];
  int pos[R];       // current position of each row (n: no row)
  unsigned live = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = w + r * G;
    pos[r] = row < n ? row : n;
    if (row < n) live |= 1u << r;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = t + k * NT;
      a[r][k] = (row < n && c <= n) ? A[(int64_t)row * g.lda + c] : T(0);
    }
  }
  for (int i = t; i < n; i += NT) rowat[i] = i;
  if (t == 0) s_ctl[3] = 0;

  // candidate of column `col` over this workgroup's live rows, published by
  // the thread that owns the column (values are in its registers)
  auto publish_cand = [&](int col) {
    if ((col % NT) != t || col >= n) return;
    const int kc = col / NT;
    uint64_t best = 0;
    int bpos = 0x7fffffff;
    T bval = T(0);
    T cv[R];  // column kc of every row: one uniform branch instead of a select chain per slot
    column_of<KC>(a, kc, cv);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const T v = cv[r];
      s_m[(col & 1) * R + r] = v;
      if (live >> r & 1u) {
        const uint64_t key = cand_key<T>(v, pos[r] == col, g.mode);
        if (key > best || (key == best && pos[r] < bpos)) {
          best = key;
          bpos = pos[r];
          bval = v;
        }
      }
    }
    s_best[col & 1] = bval;
    put16(crs, (uint32_t)(((col & 1) * G + w) * 16), best, (unsigned)bpos, (unsigned)(col + 1));
  };
  publish_cand(0);
  __syncthreads();

  bool ok = true;
  for (int i = 0; i < n; ++i) {
    const int par = i & 1;
    // ---- the pivot: wave 0 sweeps every workgroup's candidate ------------------
    if (wave == 0) {
      uint64_t bk = 0;
      unsigned bp = 0xffffffffu;
      bool good = true;
      const unsigned long long t0 = rtc();
      // every lane's (up to) 4 granules in flight at once -- lanes past G
      // read a clamped duplicate, which never changes the arg-max -- then
      // only the stale ones are re-read: one round trip per column when the
      // candidates are out, instead of one per granule
      constexpr int kQ = 4;  // G <= 256
      u32x4 v[kQ];
#pragma unroll
      for (int j = 0; j < kQ; ++j) v[j] = get16(crs, (uint32_t)((par * G + min(lane + 64 * j, G - 1)) * 16));
      for (;;) {
        bool ready = true;
#pragma unroll
        for (int j = 0; j < kQ; ++j) ready = ready && v[j].w == (unsigned)(i + 1);
        if (__ballot(!ready) == 0) break;
        if (rtc() - t0 > kSpinTicks || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
          good = false;
          break;
        }
#pragma unroll
        for (int j = 0; j < kQ; ++j)
          if (v[j].w != (unsigned)(i + 1)) v[j] = get16(crs, (uint32_t)((par * G + min(lane + 64 * j, G - 1)) * 16));
      }
#pragma unroll
      for (int j = 0; j < kQ; ++j) {
        const uint64_t k = ((uint64_t)v[j].y << 32) | v[j].x;
        if (k > bk || (k == bk && v[j].z < bp)) {
          bk = k;
          bp = v[j].z;
        }
      }
      // wave arg-max: largest key, lowest position -- two DPP ladders (the
      // 64-bit max, then the min position among its holders) instead of six
      // ds_bpermute round trips per value
      {
        const uint64_t km = dev::wave_max_u64(bk);
        bp = dev::wave_min_u32(bk == km ? bp : 0xffffffffu);
        bk = km;
      }
      const bool all_good = __ballot(!good) == 0 &&
                            __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
      if (lane == 0) {
        if (!all_good) {
          __hip_atomic_store(err, kPpErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_ctl[3] = 1;
        }
        const bool sing = bk <= 1;
        const int ppos = sing ? i : (int)bp;
        const int q = rowat[i];
        const int p = rowat[ppos];
        rowat[i] = p;
        rowat[ppos] = q;
        s_ctl[0] = p;
        s_ctl[1] = ppos;
        s_ctl[2] = sing ? 1 : 0;
      }
    }
    __syncthreads();
    if (s_ctl[3]) {
      ok = false;
      break;
    }
    const int p = s_ctl[0], ppos = s_ctl[1];
    const bool sing = s_ctl[2] != 0;
    const int q = rowat[ppos];  // the row that was at position i (now at ppos)
    const bool owner = (p % G) == w;
    const int pr = p / G;  // the pivot row's slot in its owner
    // positions: p moves to i, q (the row at position i) to ppos
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = w + r * G;
      if (row == p) {
        pos[r] = i;
        live &= ~(1u << r);
      } else if (row == q) {
        pos[r] = ppos;
      }
    }
    if (owner && t == 0) {
      g.ipiv[i] = ppos;
      g.diag[i] = sing ? 0.0 : (double)s_best[par];
      if (sing) atomicCAS(g.info, 0, i + 1);
    }
    if (sing) {
      // zero column: no interchange, no scaling, no elimination (the
      // two-kernel form's behaviour); next column's candidate
      publish_cand(i + 1);
      __syncthreads();
      continue;
    }
    // ---- the pivot row: owner scales and publishes its columns -----------------
    T u[KC];
    if (owner) {
      const T piv = s_best[par];
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int c = t + k * NT;
        T v = T(0);
#pragma unroll
        for (int r = 0; r < R; ++r) v = (r == pr) ? a[r][k] : v;
        if (c > i && c <= n) {
          v = v / piv;
          put16(rrs, (uint32_t)((par * (n + 1) + c) * 16), (uint64_t)__double_as_longlong((double)v),
                (unsigned)(i + 1), 0u);
        } else if (c == i) {
          v = T(1);
        }
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (r == pr) a[r][k] = v;
        u[k] = v;
      }
    } else {
      const unsigned long long t0 = rtc();
#pragma unroll
      for (int k = 0; k < KC; ++k) {
        const int c = t + k * NT;
        u[k] = T(0);
        if (c > i && c <= n && ok) {
          u32x4 v = get16(rrs, (uint32_t)((par * (n + 1) + c) * 16));
          while (v.z != (unsigned)(i + 1)) {
            if (rtc() - t0 > kSpinTicks || __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
              ok = false;
              break;
            }
            v = get16(rrs, (uint32_t)((par * (n + 1) + c) * 16));
          }
          u[k] = (T)__longlong_as_double((long long)(((uint64_t)v.y << 32) | v.x));
        }
      }
      if (!ok) __hip_atomic_store(err, kPpErr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- elimination of this workgroup's live rows (multipliers stay in column i)
    // column i+1 first: its owner thread then publishes the next candidate
    // before the bulk of the update
    T m[R];
#pragma unroll
    for (int r = 0; r < R; ++r) m[r] = (live >> r & 1u) ? s_m[par * R + r] : T(0);
    const int k1 = (i + 1) / NT;
    if (((i + 1) % NT) == t) {
#pragma unroll
      for (int k = 0; k < KC; ++k)
        if (k == k1)
#pragma unroll
          for (int r = 0; r < R; ++r) a[r][k] = fma(-m[r], u[k], a[r][k]);
      publish_cand(i + 1);
    }
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = t + k * NT;
      if (c > i + 1 && c <= n)
#pragma unroll
        for (int r = 0; r < R; ++r) a[r][k] = fma(-m[r], u[k], a[r][k]);
    }
    __syncthreads();  // s_m / s_best of the next parity, rowat
  }

  // ---- write-back: every row at its final position ------------------------------
  if (!ok) return;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int row = w + r * G;
    if (row >= n) continue;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const int c = t + k * NT;
      if (c <= n) A[(int64_t)pos[r] * g.lda + c] = a[r][k];
    }
  }
}

template <typename T, int NT, int R, int KC>
int launch_pp(void* A, int64_t lda, int64_t n, int mode, int* info, int* ipiv, double* diag, void* ws,
              hipStream_t s) {
  const int G = (int)((n + R - 1) / R);
  if (G > 256) return 1;  // the candidate sweep reads at most 4 granules per lane
  const size_t lds = sizeof(int) * (((size_t)n + 8 + 3) & ~(size_t)3) + sizeof(T) * (2 * R + 2);
  static const bool attr = hipFuncSetAttribute((const void*)pivot_persist_kernel<T, NT, R, KC>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024) == hipSuccess;
  if (!attr && lds > 64 * 1024) return 1;
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pivot_persist_kernel<T, NT, R, KC>, NT, lds) != hipSuccess ||
      per < 1 || !coresident(per, G))
    return 1;
  unsigned char* cand = static_cast<unsigned char*>(ws);
  unsigned char* rowb = cand + (size_t)2 * G * 16;
  // tags restart at 1 every launch: clear both buffers first (a kernel, so
  // the sequence can be graph-captured)
  GELIM_TRY(zero_async(cand, (size_t)2 * G * 16 + (size_t)2 * (n + 1) * 16, s));
  PpArgs g{A, lda, (int)n, mode, info, ipiv, diag, cand, rowb};
  hipLaunchKernelGGL((pivot_persist_kernel<T, NT, R, KC>), dim3((unsigned)G), dim3(NT), lds, s, g);
  HIP_TRY(hipGetLastError());
  return GELIM_OK;
}

}  // namespace

// Workspace bytes of pivot_persistent for order n.
size_t pivot_persist_ws_bytes(int64_t n) { return (size_t)2 * 256 * 16 + (size_t)2 * (n + 1) * 16 + 256; }

// One persistent launch of the per-pivot elimination (the two-kernel loop's
// outputs: A factored in place LAPACK-style, ipiv, diag, info).  Returns 1
// (nothing launched) when the order / device does not admit it: n > 2048, or
// the grid cannot be co-resident (GELIM_FORCE_NONPERSISTENT=1 forces that).
// Shape: 256 threads x 8 rows x 9 column slots per thread, 2048 x 2049 on 256
// CUs (512 threads x 16 rows x 5 slots on 128 CUs -- half the candidate sweep
// -- measured slower: 2048 fp64 14.0 vs 13.5 ms).
template <typename T>
int pivot_persistent(T* A, int64_t lda, int64_t n, int mode, int* info, int* ipiv, double* diag, void* ws,
                     hipStream_t s) {
  if (n > 2048 || n < 1) return 1;
  return launch_pp<T, 256, 8, 9>(A, lda, n, mode, info, ipiv, diag, ws, s);
}

template int pivot_persistent<double>(double*, int64_t, int64_t, int, int*, int*, double*, void*, hipStream_t);
template int pivot_persistent<float>(float*, int64_t, int64_t, int, int*, int*, double*, void*, hipStream_t);

}  // namespace gelim
