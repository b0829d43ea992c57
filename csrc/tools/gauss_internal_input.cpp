// gauss_internal_input — Gaussian elimination of the synthetic system
// A[i][j] = 2*min(i+1,j+1), b[i] = i.
//
// CLI parity with the reference's internal-input programs:
//   Pthreads/Version-{1,2,3}/gauss_internal_input.c, OpenMP_and_MPI/gauss_openmp/...
//   getopt "hs:t:"  ->  -s <size> (default 2048), -t <threads> (default 32), -h
//   stdout          ->  "\nMatrix Size: %d ; Threads: %d\n" (+ V2 block size,
//                       + V3 affinity line), "Application time: %f Secs"
//   timer scope     ->  initMatrix + elimination (+ back substitution), like
//                       P1i:278-284.
// New: --backend selects the parallel strategy; the default runs on the GPU.
//   --backend=hip|hip-blocked  blocked LU, fp64 MFMA trailing updates (default)
//   --backend=hip-pivot        reference per-pivot algorithm on the GPU
//   --backend=hip-rbt          randomised no-pivoting fp64 engine (butterfly
//                              transform + block LDU + fp64 refinement; falls
//                              back to the blocked LU by itself)
//   --backend=seq|omp|pthreads-v1|pthreads-v2|pthreads-v3   CPU strategies
//   --dtype=f64|f32 (f32: hip-pivot only)  --pivot=zero|partial (default zero,
//   the reference internal rule)  --verify (print B/C pairs as VERIFY=1 did)
//   --warmup=N (GPU, untimed solves first; default 1)  --affinity=yes|no (V3)
//   --no-graph  --json (one machine-readable result line)
#include <getopt.h>
#include <unistd.h>

#include <cassert>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "cli_common.h"

int main(int argc, char* argv[]) {
  int nsize = 2048, num_threads = 32;
  bool threads_given = false;
  cli::Backend backend = cli::HIP_BLOCKED;
  int dtype = 8, pivot = GELIM_PIVOT_ZERO, warmup = 1, use_graph = 1;
  bool verify = false, json = false, affinity = true;

  static option longopts[] = {{"backend", required_argument, nullptr, 'b'},
                              {"dtype", required_argument, nullptr, 'd'},
                              {"pivot", required_argument, nullptr, 'p'},
                              {"verify", no_argument, nullptr, 'v'},
                              {"json", no_argument, nullptr, 'j'},
                              {"warmup", required_argument, nullptr, 'w'},
                              {"affinity", required_argument, nullptr, 'a'},
                              {"no-graph", no_argument, nullptr, 'g'},
                              {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "hs:t:", longopts, nullptr)) != -1) {
    switch (c) {
      case 's': {
        int s = atoi(optarg);
        if (s > 0) nsize = s;
        else fprintf(stderr, "Entered size is negative, hence using the default (%d)\n", 2048);
        break;
      }
      case 't': {
        int t = atoi(optarg);
        if (t > 0) {
          num_threads = t;
          threads_given = true;
        } else {
          fprintf(stderr, "Entered number of threads is negative, hence using the default (%d)\n",
                  num_threads);
        }
        break;
      }
      case 'h':
        printf("Usage: ./program -t <num threads> -s <matrix size>"
               " [--backend=hip|hip-pivot|hip-rbt|seq|omp|pthreads-v1|pthreads-v2|pthreads-v3]"
               " [--dtype=f64|f32] [--pivot=zero|partial] [--verify] [--json]\n");
        return 0;
      case 'b':
        if (!cli::parse_backend(optarg, &backend)) {
          fprintf(stderr, "unknown backend '%s'\n", optarg);
          return -1;
        }
        break;
      case 'd': dtype = (strcmp(optarg, "f32") == 0) ? 4 : 8; break;
      case 'p': pivot = (strcmp(optarg, "partial") == 0) ? GELIM_PIVOT_PARTIAL : GELIM_PIVOT_ZERO; break;
      case 'v': verify = true; break;
      case 'j': json = true; break;
      case 'w': warmup = atoi(optarg); break;
      case 'a': affinity = (optarg[0] == 'y' || optarg[0] == '1'); break;
      case 'g': use_graph = 0; break;
      default:
        printf("Usage: ./program -t <num threads> -s <matrix size>\n");
        return -1;
    }
  }
  if (backend == cli::PTH_V3 && num_threads < 2) {
    fprintf(stderr, "Threads count should atleast be 2 for this version, hence using the default (32)\n");
    num_threads = 32;
  }
  if (backend == cli::OMP && !threads_given) {
    num_threads = gelim_cpu_max_threads();
  }
  if (dtype == 4 && backend == cli::HIP_BLOCKED) backend = cli::HIP_PIVOT;
  if (backend == cli::HIP_RBT && (verify || dtype != 8)) {
    fprintf(stderr, "hip-rbt solves a transformed fp64 system: no --verify (reference-style B), no --dtype=f32\n");
    return -1;
  }

  const int64_t n = nsize;
  if (backend == cli::PTH_V2)
    printf("\nMatrix Size: %d ; Threads: %d; Block Size: %d\n", nsize, num_threads, 16);
  else
    printf("\nMatrix Size: %d ; Threads: %d\n", nsize, num_threads);
  if (cli::is_gpu(backend) && threads_given)
    printf("note: -t %d is ignored by the GPU backends (one GPU per process; for N GPUs run "
           "`torchrun --nproc-per-node N -m gelim.cli.dist_gauss`)\n", num_threads);
  if (backend == cli::PTH_V3) {
    const long nprocs = sysconf(_SC_NPROCESSORS_ONLN);
    printf("Setting CPU Affinity : %s\n", (affinity && num_threads <= nprocs) ? "Yes" : "No");
  }

  if (cli::is_gpu(backend))
    cli::require_gpu((std::string("--backend=") + cli::backend_name(backend)).c_str(), "use --backend=omp (or seq, pthreads-v1, pthreads-v2, pthreads-v3) for the CPU engines");
  std::vector<double> B(n), C(n);
  double elapsed = 0.0;
  if (!cli::is_gpu(backend)) {
    // allocate_memory (outside the timer, P1i:276) ...
    std::vector<double> A((size_t)n * n);
    const double t0 = cli::wall();
    gelim_init_synthetic_f64(A.data(), n, B.data(), n);
    int rc = gelim_cpu_gauss(A.data(), n, B.data(), n, pivot, cli::cpu_backend_code(backend),
                             num_threads, affinity);
    if (rc == GELIM_E_SINGULAR) {
      printf("The matrix is singular\n");
      exit(-1);
    }
    if (rc != 0) cli::die("gauss");
    gelim_cpu_backsub_unit(A.data(), n, B.data(), C.data(), n);
    elapsed = cli::wall() - t0;
  } else if (backend == cli::HIP_RBT) {
    const int64_t lda = n + 1;
    double *dA = nullptr, *dx = nullptr;
    CLI_HIP(hipMalloc((void**)&dA, (size_t)(n * lda) * sizeof(double)));
    CLI_HIP(hipMalloc((void**)&dx, n * sizeof(double)));
    hipStream_t s;
    CLI_HIP(hipStreamCreate(&s));
    {
      cli::RbtSolver rbt(n, pivot, use_graph);
      auto run = [&]() {
        CLI_CHECK(gelim_gpu_init_synthetic(dA, lda, n, s));
        rbt.solve(dA, lda, dx, s);
        CLI_HIP(hipStreamSynchronize(s));
      };
      for (int w = 0; w < warmup; ++w) run();
      const double t0 = cli::wall();
      run();
      elapsed = cli::wall() - t0;
      const int info = rbt.info(s);
      if (info > 0) {
        printf("The matrix is singular\n");
        exit(-1);
      }
      if (info < 0) cli::die("plan_info");
      CLI_HIP(hipMemcpy(C.data(), dx, n * sizeof(double), hipMemcpyDeviceToHost));
      printf("Device: %s ; Backend: %s ; dtype: f64\n", cli::device_name().c_str(), cli::backend_name(backend));
      rbt.note();
    }
    (void)hipFree(dA);
    (void)hipFree(dx);
    (void)hipStreamDestroy(s);
  } else {
    const int algo = backend == cli::HIP_BLOCKED ? GELIM_GPU_BLOCKED : GELIM_GPU_PIVOT;
    gelim_gauss_plan* plan = gelim_gauss_plan_create(n, algo, pivot, dtype, use_graph);
    if (!plan) cli::die("plan_create");
    const int64_t lda = gelim_gauss_plan_lda(plan);
    void* dA = nullptr;
    double *dx = nullptr, *dbn = nullptr;
    CLI_HIP(hipMalloc(&dA, (size_t)(n * lda * dtype)));
    CLI_HIP(hipMalloc((void**)&dx, n * sizeof(double)));
    CLI_HIP(hipMalloc((void**)&dbn, n * sizeof(double)));
    hipStream_t s;
    CLI_HIP(hipStreamCreate(&s));
    auto run = [&]() {
      if (dtype == 8) CLI_CHECK(gelim_gpu_init_synthetic(static_cast<double*>(dA), lda, n, s));
      else CLI_CHECK(gelim_gpu_init_synthetic_f32(static_cast<float*>(dA), lda, n, s));
      CLI_CHECK(gelim_gauss_plan_solve(plan, dA, lda, dx, verify ? dbn : nullptr, s));
      CLI_HIP(hipStreamSynchronize(s));
    };
    for (int w = 0; w < warmup; ++w) run();
    const double t0 = cli::wall();
    run();
    elapsed = cli::wall() - t0;
    // > 0: 1 + the first zero-pivot column; < 0: a GPU error (hand-off
    // timeout, corrupt row map ...), never reported as "singular"
    const int info = gelim_gauss_plan_info(plan, s);
    if (info > 0) {
      printf("The matrix is singular\n");
      exit(-1);
    }
    if (info < 0) cli::die("plan_info");
    CLI_HIP(hipMemcpy(C.data(), dx, n * sizeof(double), hipMemcpyDeviceToHost));
    if (verify) CLI_HIP(hipMemcpy(B.data(), dbn, n * sizeof(double), hipMemcpyDeviceToHost));
    printf("Device: %s ; Backend: %s ; dtype: %s\n", cli::device_name().c_str(),
           cli::backend_name(backend), dtype == 8 ? "f64" : "f32");
    gelim_gauss_plan_destroy(plan);
    (void)hipFree(dA);
    (void)hipFree(dx);
    (void)hipFree(dbn);
    (void)hipStreamDestroy(s);
  }

  printf("Application time: %f Secs\n", elapsed);
  if (verify)
    for (int64_t i = 0; i < n; i++) printf("%6.5f %5.5f\n", B[i], C[i]);
  if (json) {
    // max |C - exact| with exact = (-0.5, 0, ..., 0, 0.5)
    double err = 0.0;
    for (int64_t i = 0; i < n; ++i) {
      double ex = (n == 1) ? 0.0 : (i == 0 ? -0.5 : (i == n - 1 ? 0.5 : 0.0));
      if (n == 1) ex = 0.0;
      double e = std::abs(C[i] - ex);
      if (e > err) err = e;
    }
    const std::string thr = cli::is_gpu(backend) ? "null" : std::to_string(num_threads);
    printf("{\"program\": \"gauss_internal_input\", \"n\": %lld, \"backend\": \"%s\", "
           "\"threads\": %s, \"gpus\": %d, \"dtype\": \"%s\", \"time_s\": %.9f, \"gflops\": %.3f, "
           "\"max_abs_err\": %.3e}\n",
           (long long)n, cli::backend_name(backend), thr.c_str(), cli::is_gpu(backend) ? 1 : 0,
           dtype == 8 ? "f64" : "f32", elapsed, (2.0 / 3.0) * (double)n * n * n / elapsed * 1e-9, err);
  }
  return 0;
}
