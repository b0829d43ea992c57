// Random butterfly transform (RBT) group matrices, shared by the single-GPU
// randomised engine (lu_mixed.hip) and its distributed form (dist_rbt.hip).
//
// Depth-2 recursive butterfly W = L1 L0 on an order-np index space (np a
// multiple of 4, h = np / 4): L0 = B<np> = 1/sqrt2 [R S; R -S] on (i, i + np/2),
// L1 = diag(B<np/2>_a, B<np/2>_b) on (i, i + h) and (i + 2h, i + 3h); R, S
// diagonal with entries exp(r / 10), r uniform in [-1/2, 1/2].  Both levels
// act on the index group {i, i + h, i + 2h, i + 3h} as one 4 x 4 matrix W_i,
// so U^T A V is one pass over A: every 4 x 4 group of entries becomes
// U_i^T A_g V_j.
#pragma once

#include <hip/hip_runtime.h>

namespace gelim {
namespace rbt {

// d: 8 arrays of h doubles: R0[i], R0[i+h], S0[i], S0[i+h], Ra[i], Sa[i], Rb[i], Sb[i]
__device__ __forceinline__ void group_w(const double* __restrict__ d, int h, int i, double (&W)[4][4]) {
  const double r0 = d[i], r0h = d[h + i], s0 = d[2 * h + i], s0h = d[3 * h + i];
  const double ra = d[4 * h + i], sa = d[5 * h + i], rb = d[6 * h + i], sb = d[7 * h + i];
  // L0 (order i, i+h, i+2h, i+3h)
  const double L0[4][4] = {{r0, 0, s0, 0}, {0, r0h, 0, s0h}, {r0, 0, -s0, 0}, {0, r0h, 0, -s0h}};
  const double L1[4][4] = {{ra, sa, 0, 0}, {ra, -sa, 0, 0}, {0, 0, rb, sb}, {0, 0, rb, -sb}};
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      double v = 0.0;
#pragma unroll
      for (int c = 0; c < 4; ++c) v += L1[a][c] * L0[c][b];
      W[a][b] = 0.5 * v;  // (1/sqrt2)^2
    }
}

}  // namespace rbt
}  // namespace gelim
