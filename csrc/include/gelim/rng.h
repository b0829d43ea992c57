// Counter-based uniform generator shared by host C++ and HIP device code so
// that a random system built on the GPU is bit-identical to the host one.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GELIM_HD __host__ __device__ __forceinline__
#else
#define GELIM_HD inline
#endif

namespace gelim {

GELIM_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// U[-1, 1) with 53 random bits, keyed by (seed, i, j).
GELIM_HD double rng_uniform_pm1(uint64_t seed, int64_t i, int64_t j) {
  uint64_t k = splitmix64(seed ^ splitmix64(((uint64_t)i << 32) ^ (uint64_t)j));
  return (double)(k >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

}  // namespace gelim
