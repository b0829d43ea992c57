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

// ---- DPP wave reductions (gfx9-family row_shr / row_bcast scans) ---------
// The classic inclusive-scan ladder: row_shr:1,2,4,8 inside each 16-lane row,
// then row_bcast:15 and row_bcast:31 across rows; lane 63 ends with the
// reduction of all 64 lanes and is read with v_readlane into a uniform value.
// ~6 dependent VALU+DPP steps instead of 6 ds_bpermute round trips per value.
enum : int {
  kDppRowShr1 = 0x111,
  kDppRowShr2 = 0x112,
  kDppRowShr4 = 0x114,
  kDppRowShr8 = 0x118,
  kDppRowBcast15 = 0x142,
  kDppRowBcast31 = 0x143
};

template <int CTRL, int ROW_MASK, int BANK_MASK>
__device__ __forceinline__ unsigned dpp_u32(unsigned identity, unsigned v) {
  // lanes whose source is out of range (or masked) keep `identity`
  return (unsigned)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROW_MASK, BANK_MASK, false);
}

// 64-bit unsigned max over the wave (identity 0); result uniform.
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
  unsigned hi = (unsigned)(v >> 32), lo = (unsigned)v;
#define GELIM_MAX_STEP(CTRL, RM, BM)                                     \
  {                                                                      \
    const unsigned h2 = dpp_u32<CTRL, RM, BM>(0u, hi);                   \
    const unsigned l2 = dpp_u32<CTRL, RM, BM>(0u, lo);                   \
    const bool gt = (h2 > hi) || (h2 == hi && l2 > lo);                  \
    hi = gt ? h2 : hi;                                                   \
    lo = gt ? l2 : lo;                                                   \
  }
  GELIM_MAX_STEP(kDppRowShr1, 0xf, 0xf)
  GELIM_MAX_STEP(kDppRowShr2, 0xf, 0xf)
  GELIM_MAX_STEP(kDppRowShr4, 0xf, 0xf)
  GELIM_MAX_STEP(kDppRowShr8, 0xf, 0xf)
  GELIM_MAX_STEP(kDppRowBcast15, 0xa, 0xf)
  GELIM_MAX_STEP(kDppRowBcast31, 0xc, 0xf)
#undef GELIM_MAX_STEP
  hi = (unsigned)__builtin_amdgcn_readlane((int)hi, 63);
  lo = (unsigned)__builtin_amdgcn_readlane((int)lo, 63);
  return ((uint64_t)hi << 32) | lo;
}

// 32-bit unsigned max over the wave (identity 0); result uniform.
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
  v = max(v, dpp_u32<kDppRowShr1, 0xf, 0xf>(0u, v));
  v = max(v, dpp_u32<kDppRowShr2, 0xf, 0xf>(0u, v));
  v = max(v, dpp_u32<kDppRowShr4, 0xf, 0xf>(0u, v));
  v = max(v, dpp_u32<kDppRowShr8, 0xf, 0xf>(0u, v));
  v = max(v, dpp_u32<kDppRowBcast15, 0xa, 0xf>(0u, v));
  v = max(v, dpp_u32<kDppRowBcast31, 0xc, 0xf>(0u, v));
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// 32-bit unsigned min over the wave (identity 0xffffffff); result uniform.
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
  v = min(v, dpp_u32<kDppRowShr1, 0xf, 0xf>(0xffffffffu, v));
  v = min(v, dpp_u32<kDppRowShr2, 0xf, 0xf>(0xffffffffu, v));
  v = min(v, dpp_u32<kDppRowShr4, 0xf, 0xf>(0xffffffffu, v));
  v = min(v, dpp_u32<kDppRowShr8, 0xf, 0xf>(0xffffffffu, v));
  v = min(v, dpp_u32<kDppRowBcast15, 0xa, 0xf>(0xffffffffu, v));
  v = min(v, dpp_u32<kDppRowBcast31, 0xc, 0xf>(0xffffffffu, v));
  return (unsigned)__builtin_amdgcn_readlane((int)v, 63);
}

// Write-through (sc1) stores through a buffer resource.  Bulk results written
// this way leave no dirty lines in the XCD's L2, so the kernel-end release
// has nothing to write back: a dependent kernel boundary costs ~1.5 us plus
// B / 6 TB/s for B dirty bytes (MI355X_MICROARCH.md, "boundary"), i.e. ~5 us
// behind a trailing update of a 2048^2 fp64 matrix.  The store itself is
// issued like any other and overlaps the kernel's remaining work.
typedef unsigned wt_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint64_t bytes) {
  const uint32_t n = bytes > 0xffffffffull ? 0xffffffffu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}
__device__ __forceinline__ void store_wt(__amdgpu_buffer_rsrc_t r, uint32_t byte_off, double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const wt_u32x2 x = {(unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(x, r, (int)byte_off, 0, 16 /* sc1 */);
}

// Plain 8-byte buffer store: the per-thread part of the address is one 32-bit
// VGPR and the uniform part an SGPR / immediate, so a run of stores to
// different columns of a column-major buffer costs one instruction each
// (global stores need a 64-bit address add per store).
__device__ __forceinline__ void store_buf(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const wt_u32x2 x = {(unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(x, r, (int)voff, (int)soff, 0);
}

// The same with sc1 (write-through): for payloads another workgroup of the
// same launch reads (lu_panel.hip fused narrow update).
__device__ __forceinline__ void store_buf_wt(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, double v) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const wt_u32x2 x = {(unsigned)b, (unsigned)(b >> 32)};
  __builtin_amdgcn_raw_buffer_store_b64(x, r, (int)voff, (int)soff, 16 /* sc1 */);
}

// Masked load without control flow: p must be a valid address (callers
// clamp their indices), the value is selected afterwards.  Written as
// `ok ? p[i] : 0`, LLVM turns each masked load into an exec-masked branch
// that ends in its own s_waitcnt vmcnt(0) — independent loads then run one
// after another instead of being in flight together.
template <typename T>
__device__ __forceinline__ T load_sel(const T* p, bool ok, T dflt = T(0)) {
  const T v = *p;
  return ok ? v : dflt;
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

// Pivot key as an order-preserving unsigned integer: 0 = no candidate,
// larger = better.  PARTIAL: bits(|a|)+1 (non-negative doubles order like
// their bit patterns; NaN never wins); ZERO: 3 diag non-zero, 2 other non-zero,
// 1 zero.
template <typename T>
__device__ __forceinline__ uint64_t pivot_ukey(T a, bool is_diag, int mode) {
  if (mode == 1) {
    const double v = fabs((double)a);
    if (v != v) return 0;
    return (uint64_t)__double_as_longlong(v) + 1;
  }
  if (a == T(0)) return 1;
  return is_diag ? 3 : 2;
}

// Branchless pivot key for a compile-time rule (MODE 1 = PARTIAL, 0 = ZERO):
// 0 = not a candidate; every live row has a key >= 1 (NaN ranks as zero).
template <int MODE>
__device__ __forceinline__ uint64_t pivot_ukey_t(double a, bool is_diag, bool ok) {
  if constexpr (MODE == 1) {
    const uint64_t bits = (uint64_t)__double_as_longlong(a) & 0x7fffffffffffffffull;
    const bool nan = bits > 0x7ff0000000000000ull;  // ranks like zero: a live row always wins
    return ok ? (nan ? 1 : bits + 1) : 0;
  } else {
    const uint64_t k = (a == 0.0) ? 1 : (is_diag ? 3 : 2);
    return ok ? k : 0;
  }
}

}  // namespace dev
}  // namespace gelim
