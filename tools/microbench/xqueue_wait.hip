// Cross-queue event semantics on gfx950 / ROCm 7.2, as the DistributedRBT
// executor relies on them (csrc/hip/drbt_exec.hip): when does a kernel on
// stream Y, made to wait (hipStreamWaitEvent) for an event recorded on
// stream X between X's kernels K1 and K2, start -- after K1 (the event's
// position) or after K2 (X's tail)?  And does stream X's own later work wait
// for Y when Y waits on X?  Each kernel spins for a fixed time (s_memrealtime,
// 100 MHz) and stamps its start and end; non-blocking streams.
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/microbench/xqueue_wait.hip -o /tmp/xqueue_wait
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                           \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__global__ void spin(unsigned long long* st, int slot, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long t = t0;
  while (t - t0 < ticks) t = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    st[2 * slot] = t0;
    st[2 * slot + 1] = t;
  }
}

int main() {
  unsigned long long *st, h[32];
  CHECK(hipMalloc(&st, sizeof(h)));
  hipStream_t X, Y;
  CHECK(hipStreamCreateWithFlags(&X, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&Y, hipStreamNonBlocking));
  hipEvent_t E;
  CHECK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
  auto us = [&](int slot, int which) { return (double)(h[2 * slot + which] - h[0]) / 100.0; };
  auto rel = [&](int slot, int which) { return ((double)h[2 * slot + which] - (double)h[8]) / 100.0; };
  hipStream_t Z;
  CHECK(hipStreamCreateWithFlags(&Z, hipStreamNonBlocking));
  hipEvent_t E0;
  CHECK(hipEventCreateWithFlags(&E0, hipEventDisableTiming));
  for (int variant = 0; variant < 6; ++variant) {
    for (int rep = 0; rep < 3; ++rep) {
      CHECK(hipMemset(st, 0, sizeof(h)));
      CHECK(hipDeviceSynchronize());
      const unsigned long long T1 = 2000, T2 = 5000, T3 = 500;  // 20 us, 50 us, 5 us
      if (variant == 0) {  // X: K1, rec E, K2; then Y: wait E, K3
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 0, T1);
        CHECK(hipEventRecord(E, X));
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 1, T2);
        CHECK(hipStreamWaitEvent(Y, E, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 2, T3);
      } else if (variant == 1) {  // X: K1, rec E; Y: wait E, K3; X: K2
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 0, T1);
        CHECK(hipEventRecord(E, X));
        CHECK(hipStreamWaitEvent(Y, E, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 2, T3);
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 1, T2);
      } else if (variant == 2) {  // X: K1, rec E; Y: wait E, K2 (long); X: K3 -- does K3 wait for Y?
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 0, T1);
        CHECK(hipEventRecord(E, X));
        CHECK(hipStreamWaitEvent(Y, E, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 1, T2);
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 2, T3);
      } else if (variant >= 4) {  // Z: K0 (20 us), rec E0; X: wait E0, K1 (20 us), rec E, K2 (50 us); Y: wait E, K3
        hipLaunchKernelGGL(spin, 1, 64, 0, Z, st, 4, T1);
        CHECK(hipEventRecord(E0, Z));
        CHECK(hipStreamWaitEvent(X, E0, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 0, T1);
        CHECK(hipEventRecord(E, X));
        if (variant == 5) (void)hipEventQuery(E);  // a flush after the record?
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 1, T2);
        CHECK(hipStreamWaitEvent(Y, E, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 2, T3);
      } else {  // X: K1 (long), rec E; Y: K2 (short); Y: wait E ... and X: K3 after; when does X's K3 start
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 0, T1);
        CHECK(hipEventRecord(E, X));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 1, T3);
        CHECK(hipStreamWaitEvent(Y, E, 0));
        hipLaunchKernelGGL(spin, 1, 64, 0, Y, st, 3, T3);
        hipLaunchKernelGGL(spin, 1, 64, 0, X, st, 2, T2);
      }
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemcpy(h, st, sizeof(h), hipMemcpyDeviceToHost));
      if (variant == 0)
        std::printf("v0 X:K1,rec,K2 then Y:wait,K3  K1 %.1f-%.1f K2 %.1f-%.1f  K3 starts %.1f us\n", us(0, 0), us(0, 1),
                    us(1, 0), us(1, 1), us(2, 0));
      else if (variant == 1)
        std::printf("v1 X:K1,rec; Y:wait,K3; X:K2  K1 %.1f-%.1f K2 %.1f-%.1f  K3 starts %.1f us\n", us(0, 0), us(0, 1),
                    us(1, 0), us(1, 1), us(2, 0));
      else if (variant == 2)
        std::printf("v2 X:K1,rec; Y:wait,K2(50us); X:K3  K1 %.1f-%.1f  Y.K2 %.1f-%.1f  X.K3 starts %.1f us\n", us(0, 0),
                    us(0, 1), us(1, 0), us(1, 1), us(2, 0));
      else if (variant >= 4)
        std::printf("v%d Z:K0,rec0; X:wait0,K1,rec,K2; Y:wait,K3%s  K0 %.1f-%.1f K1 %.1f-%.1f K2 %.1f-%.1f  K3 starts %.1f us\n",
                    variant, variant == 5 ? " (+query)" : "", rel(4, 0), rel(4, 1), rel(0, 0), rel(0, 1), rel(1, 0),
                    rel(1, 1), rel(2, 0));
      else
        std::printf("v3 X:K1,rec; Y:K2,wait,K4; X:K3(50us)  K1 %.1f-%.1f  Y.K4 starts %.1f  X.K3 %.1f-%.1f us\n",
                    us(0, 0), us(0, 1), us(3, 0), us(2, 0), us(2, 1));
    }
  }
  return 0;
}
