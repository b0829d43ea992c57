// hip_matmul — fp32 C = A * B on the GPU vs the sequential and OpenMP CPU
// loops (CLI parity with CUDA_and_OpenMP/Version-{1,2}/cuda_matmul.cu).
//
//   usage   ->  hip_matmul <array size> [--kernel=mfma|naive-row|naive-elem]
//               [--no-seq] [--no-omp] [--threads=N] [--verify] [--json]
//               [--warmup=N] [--chunks=N]
//   stdout  ->  "GPU Time: <s>", "Seq (vectorized) Time: <s>", "OMP Time: <s>"
//               (std::cout default formatting, CU2:166,173,180), plus
//               "GPU Kernel Time: <s>".
//   GPU Time keeps the reference semantics: malloc + H2D + kernel + D2H +
//   free, all inside the timer (CU2:135-165).  Host arrays are pinned
//   (allocated outside the timer, like the reference's `new float[]`).
// --chunks=N (default 1 = the reference's serial copies; N > 1) overlaps the
// transfers with the GEMM inside the same timer scope: B then A in N row
// chunks on an upload stream, each chunk's rows of C multiplied as soon as
// it lands and copied back on a download stream (PCIe is full duplex).
// Measured at 2048 (profiles/hip_matmul_2048_cli.txt): 1.66 ms serial, 1.82 ms
// with 2 chunks, 2.08 ms with 4 — in this program the async copies and the
// extra small GEMMs cost more than the overlap saves (hipMalloc/hipFree inside
// the timer dominate), so serial is the default.
// Unlike the reference the GPU result is verified (--verify) against the
// CPU result with a relative tolerance (its verify() was never called and its
// absolute 1e-4 could not pass).
#include <getopt.h>

#include <algorithm>
#include <cmath>
#include <iostream>
#include <string>
#include <vector>

#include "cli_common.h"

int main(int argc, char* argv[]) {
  int kernel = GELIM_MM_MFMA, threads = 0, warmup = 1, chunks = 1;
  bool do_seq = true, do_omp = true, verify = false, json = false;
  static option longopts[] = {{"kernel", required_argument, nullptr, 'k'},
                              {"no-seq", no_argument, nullptr, 's'},
                              {"no-omp", no_argument, nullptr, 'o'},
                              {"threads", required_argument, nullptr, 't'},
                              {"verify", no_argument, nullptr, 'v'},
                              {"json", no_argument, nullptr, 'j'},
                              {"warmup", required_argument, nullptr, 'w'},
                              {"chunks", required_argument, nullptr, 'c'},
                              {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "", longopts, nullptr)) != -1) {
    switch (c) {
      case 'k':
        if (!strcmp(optarg, "naive-row") || !strcmp(optarg, "v1")) kernel = GELIM_MM_NAIVE_ROW;
        else if (!strcmp(optarg, "naive-elem") || !strcmp(optarg, "v2")) kernel = GELIM_MM_NAIVE_ELEM;
        else kernel = GELIM_MM_MFMA;
        break;
      case 's': do_seq = false; break;
      case 'o': do_omp = false; break;
      case 't': threads = atoi(optarg); break;
      case 'v': verify = true; break;
      case 'j': json = true; break;
      case 'w': warmup = atoi(optarg); break;
      case 'c': chunks = std::max(1, atoi(optarg)); break;
      default: break;
    }
  }
  if (argc - optind < 1) {
    std::cout << "Invalid number of arguments: usage " << argv[0] << " <array size>" << std::endl;
    exit(0);
  }
  const int64_t nsize = std::atoll(argv[optind]);
  if (nsize <= 0) {
    std::cout << "Invalid array size" << std::endl;
    exit(0);
  }
  cli::require_gpu("hip_matmul (GPU Time)", "the sequential / OpenMP loops alone are not a mode of this program");
  const size_t elems = (size_t)nsize * nsize;
  const size_t bytes = elems * sizeof(float);
  float *A, *B, *C;
  CLI_HIP(hipHostMalloc((void**)&A, bytes, hipHostMallocDefault));
  CLI_HIP(hipHostMalloc((void**)&B, bytes, hipHostMallocDefault));
  CLI_HIP(hipHostMalloc((void**)&C, bytes, hipHostMallocDefault));
  gelim_init_matmul_f32(A, B, nsize);

  chunks = (int)std::min<int64_t>(chunks, nsize);
  hipStream_t up = nullptr, comp = nullptr, down = nullptr;
  std::vector<hipEvent_t> landed(chunks), k0(chunks), k1(chunks);
  if (chunks > 1) {
    CLI_HIP(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
    CLI_HIP(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
    CLI_HIP(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
    for (int i = 0; i < chunks; ++i) {
      CLI_HIP(hipEventCreateWithFlags(&landed[i], hipEventDisableTiming));
      CLI_HIP(hipEventCreate(&k0[i]));
      CLI_HIP(hipEventCreate(&k1[i]));
    }
  }
  auto gpu_run_pipelined = [&](double* kernel_s) {
    float *dA, *dB, *dC;
    CLI_HIP(hipMalloc((void**)&dA, bytes));
    CLI_HIP(hipMalloc((void**)&dB, bytes));
    CLI_HIP(hipMalloc((void**)&dC, bytes));
    CLI_HIP(hipMemcpyAsync(dB, B, bytes, hipMemcpyHostToDevice, up));
    for (int i = 0; i < chunks; ++i) {
      const int64_t r0 = nsize * i / chunks, r1 = nsize * (i + 1) / chunks;
      const size_t off = (size_t)r0 * nsize, cb = (size_t)(r1 - r0) * nsize * sizeof(float);
      CLI_HIP(hipMemcpyAsync(dA + off, A + off, cb, hipMemcpyHostToDevice, up));
      CLI_HIP(hipEventRecord(landed[i], up));
      CLI_HIP(hipStreamWaitEvent(comp, landed[i], 0));
      CLI_HIP(hipEventRecord(k0[i], comp));
      CLI_CHECK(gelim_gpu_matmul_f32(dA + off, dB, dC + off, r1 - r0, nsize, nsize, kernel, comp));
      CLI_HIP(hipEventRecord(k1[i], comp));
      CLI_HIP(hipStreamWaitEvent(down, k1[i], 0));
      CLI_HIP(hipMemcpyAsync(C + off, dC + off, cb, hipMemcpyDeviceToHost, down));
    }
    CLI_HIP(hipStreamSynchronize(down));
    CLI_HIP(hipDeviceSynchronize());
    double ks = 0.0;
    for (int i = 0; i < chunks; ++i) {
      float ms = 0.f;
      CLI_HIP(hipEventElapsedTime(&ms, k0[i], k1[i]));
      ks += ms * 1e-3;
    }
    *kernel_s = ks;
    CLI_HIP(hipFree(dA));
    CLI_HIP(hipFree(dB));
    CLI_HIP(hipFree(dC));
  };
  auto gpu_run = [&](double* kernel_s) {
    if (chunks > 1) return gpu_run_pipelined(kernel_s);
    float *dA, *dB, *dC;
    CLI_HIP(hipMalloc((void**)&dA, bytes));
    CLI_HIP(hipMalloc((void**)&dB, bytes));
    CLI_HIP(hipMalloc((void**)&dC, bytes));
    CLI_HIP(hipMemcpy(dA, A, bytes, hipMemcpyHostToDevice));
    CLI_HIP(hipMemcpy(dB, B, bytes, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CLI_HIP(hipEventCreate(&e0));
    CLI_HIP(hipEventCreate(&e1));
    CLI_HIP(hipEventRecord(e0, 0));
    CLI_CHECK(gelim_gpu_matmul_f32(dA, dB, dC, nsize, nsize, nsize, kernel, nullptr));
    CLI_HIP(hipEventRecord(e1, 0));
    CLI_HIP(hipDeviceSynchronize());
    CLI_HIP(hipMemcpy(C, dC, bytes, hipMemcpyDeviceToHost));
    float ms = 0.f;
    CLI_HIP(hipEventElapsedTime(&ms, e0, e1));
    *kernel_s = ms * 1e-3;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    CLI_HIP(hipFree(dA));
    CLI_HIP(hipFree(dB));
    CLI_HIP(hipFree(dC));
  };
  double ks = 0.0;
  for (int w = 0; w < warmup; ++w) gpu_run(&ks);
  const double g0 = cli::wall();
  gpu_run(&ks);
  const double gpu_s = cli::wall() - g0;
  std::cout << "GPU Time: " << gpu_s << '\n';
  std::cout << "GPU Kernel Time: " << ks << '\n';

  std::vector<float> Cgpu;
  if (verify) Cgpu.assign(C, C + elems);

  double seq_s = -1, omp_s = -1;
  if (do_seq) {
    const double t0 = cli::wall();
    gelim_cpu_matmul_f32(A, B, C, nsize, 0, 0);
    seq_s = cli::wall() - t0;
    std::cout << "Seq (vectorized) Time: " << seq_s << '\n';
  }
  if (do_omp) {
    const double t0 = cli::wall();
    gelim_cpu_matmul_f32(A, B, C, nsize, 1, threads);
    omp_s = cli::wall() - t0;
    std::cout << "OMP Time: " << omp_s << '\n';
  }
  double max_rel = 0.0;
  if (verify) {
    if (!do_seq && !do_omp) gelim_cpu_matmul_f32(A, B, C, nsize, 1, threads);
    for (size_t i = 0; i < elems; ++i) {
      const double ref = C[i], got = Cgpu[i];
      const double rel = std::fabs(got - ref) / std::max(1e-30, std::fabs(ref));
      max_rel = std::max(max_rel, rel);
    }
    std::cout << "Verify max rel err: " << max_rel << (max_rel < 1e-3 ? " (PASS)" : " (FAIL)")
              << '\n';
  }
  if (json) {
    const double flops = 2.0 * (double)nsize * nsize * nsize;
    char rel_buf[32];
    snprintf(rel_buf, sizeof(rel_buf), "%.3e", max_rel);
    const std::string rel_str = rel_buf;
    printf("{\"program\": \"hip_matmul\", \"n\": %lld, \"kernel\": %d, \"gpu_time_s\": %.9f, "
           "\"gpu_kernel_s\": %.9f, \"kernel_tflops\": %.3f, \"seq_time_s\": %.6f, "
           "\"omp_time_s\": %.6f, \"speedup_vs_seq\": %.3f, \"kernel_speedup_vs_seq\": %.3f, "
           "\"max_rel_err\": %s}\n",
           (long long)nsize, kernel, gpu_s, ks, flops / ks * 1e-12, seq_s, omp_s,
           seq_s > 0 ? seq_s / gpu_s : -1.0, seq_s > 0 ? seq_s / ks : -1.0,
           verify ? rel_str.c_str() : "null");  // null: not verified (no --verify)
  }
  (void)hipHostFree(A);
  (void)hipHostFree(B);
  (void)hipHostFree(C);
  return 0;
}
