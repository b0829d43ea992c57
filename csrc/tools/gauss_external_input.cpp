// gauss_external_input — Gaussian elimination of a system read from a
// reference `.dat` coordinate file, with the preset solution X__ = (1..n)
// and R = A * X__.
//
// CLI parity:
//   usage           ->  <matrixfile> [threads]
//   stdout          ->  "\nMatrix File: %s; Matrix Size: %d ; Threads: %d\n"
//                       (the correct n, as the OpenMP version prints it;
//                       V2 adds "; Block Size: 16", V3 the affinity line),
//                       "Time:  %f seconds", "Error: %e"
//   timer scope     ->  elimination only on the CPU backends (P1e:300-302);
//                       elimination + back substitution on the GPU ones.
//   pivoting        ->  partial (argmax |a|), as every external program does.
// Options as gauss_internal_input (--backend, --warmup, --json, --no-graph,
// --affinity); the default backend is the GPU blocked LU (fp64).
#include <getopt.h>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "cli_common.h"

int main(int argc, char* argv[]) {
  cli::Backend backend = cli::HIP_BLOCKED;
  int warmup = 1, use_graph = 1;
  bool json = false, affinity = true;
  static option longopts[] = {{"backend", required_argument, nullptr, 'b'},
                              {"json", no_argument, nullptr, 'j'},
                              {"warmup", required_argument, nullptr, 'w'},
                              {"affinity", required_argument, nullptr, 'a'},
                              {"no-graph", no_argument, nullptr, 'g'},
                              {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "", longopts, nullptr)) != -1) {
    switch (c) {
      case 'b':
        if (!cli::parse_backend(optarg, &backend)) {
          fprintf(stderr, "unknown backend '%s'\n", optarg);
          return -1;
        }
        break;
      case 'j': json = true; break;
      case 'w': warmup = atoi(optarg); break;
      case 'a': affinity = (optarg[0] == 'y' || optarg[0] == '1'); break;
      case 'g': use_graph = 0; break;
      default:
        fprintf(stderr, "usage: %s <matrixfile> <number_of_threads (optional)>\n", argv[0]);
        exit(-1);
    }
  }
  const int npos = argc - optind;
  if (npos != 1 && npos != 2) {
    fprintf(stderr, "usage: %s <matrixfile> <number_of_threads (optional)>\n", argv[0]);
    exit(-1);
  }
  const char* fname = argv[optind];
  int num_threads = (backend == cli::OMP) ? gelim_cpu_max_threads() : 32;
  if (npos == 2) {
    const int t = atoi(argv[optind + 1]);
    if (t <= 0) {
      fprintf(stderr, "Error: Number of threads must be a postive integer.\n");
      fprintf(stderr, "usage: %s <matrixfile> <number_of_threads (optional)>\n", argv[0]);
      exit(-1);
    }
    if (backend == cli::PTH_V3 && t < 2) {
      fprintf(stderr, "Error: Number of threads must atleast be 2 for this version.\n");
      exit(-1);
    }
    num_threads = t;
  }

  const int64_t nsize = gelim_dat_size(fname);
  if (nsize <= 0) {
    fprintf(stderr, "The matrix file open error\n");
    exit(-1);
  }
  const int64_t n = nsize;
  if (backend == cli::PTH_V2)
    printf("\nMatrix File: %s; Matrix Size: %lld ; Threads: %d; Block Size: %d\n", fname,
           (long long)n, num_threads, 16);
  else
    printf("\nMatrix File: %s; Matrix Size: %lld ; Threads: %d\n", fname, (long long)n,
           num_threads);
  if (backend == cli::PTH_V3) {
    const long nprocs = sysconf(_SC_NPROCESSORS_ONLN);
    printf("Setting CPU Affinity : %s\n", (affinity && num_threads <= nprocs) ? "Yes" : "No");
  }
  if (cli::is_gpu(backend) && npos == 2)
    printf("note: the thread count %d is ignored by the GPU backends (one GPU per process; for N GPUs run "
           "`torchrun --nproc-per-node N -m gelim.cli.dist_gauss --file <matrix>`)\n", num_threads);

  // initMatrix + initRHS on the host, in the reference's order (P1e:296-297)
  const bool gpu = cli::is_gpu(backend);
  if (gpu) cli::require_gpu((std::string("--backend=") + cli::backend_name(backend)).c_str(), "use --backend=omp (or seq, pthreads-v1, pthreads-v2, pthreads-v3) for the CPU engines");
  const int64_t lda = gpu ? n + 1 : n;  // GPU: augmented [A | R]
  std::vector<double> A((size_t)n * lda), R(n), X(n);
  if (gelim_dat_read(fname, A.data(), n, lda) != 0) cli::die("dat_read");
  gelim_init_rhs_f64(A.data(), lda, R.data(), n);

  double elapsed = 0.0;
  if (!gpu) {
    const double t0 = cli::wall();
    const int rc = gelim_cpu_gauss(A.data(), lda, R.data(), n, GELIM_PIVOT_PARTIAL,
                                   cli::cpu_backend_code(backend), num_threads, affinity);
    elapsed = cli::wall() - t0;
    if (rc == GELIM_E_SINGULAR) {
      fprintf(stderr, "The matrix is singular\n");
      exit(-1);
    }
    if (rc != 0) cli::die("gauss");
    gelim_cpu_backsub_unit(A.data(), lda, R.data(), X.data(), n);
  } else {
    for (int64_t i = 0; i < n; ++i) A[i * lda + n] = R[i];
    if (backend == cli::HIP_RBT) {
      double *dA = nullptr, *dx = nullptr;
      CLI_HIP(hipMalloc((void**)&dA, A.size() * sizeof(double)));
      CLI_HIP(hipMalloc((void**)&dx, n * sizeof(double)));
      CLI_HIP(hipMemcpy(dA, A.data(), A.size() * sizeof(double), hipMemcpyHostToDevice));
      hipStream_t s;
      CLI_HIP(hipStreamCreate(&s));
      {
        cli::RbtSolver rbt(n, GELIM_PIVOT_PARTIAL, use_graph);
        auto run = [&]() {
          rbt.solve(dA, lda, dx, s);
          CLI_HIP(hipStreamSynchronize(s));
        };
        for (int w = 0; w < warmup; ++w) run();
        const double t0 = cli::wall();
        run();
        elapsed = cli::wall() - t0;
        const int info = rbt.info(s);
        if (info > 0) {
          fprintf(stderr, "The matrix is singular\n");
          exit(-1);
        }
        if (info < 0) cli::die("plan_info");
        CLI_HIP(hipMemcpy(X.data(), dx, n * sizeof(double), hipMemcpyDeviceToHost));
        printf("Device: %s ; Backend: %s ; dtype: f64\n", cli::device_name().c_str(), cli::backend_name(backend));
        rbt.note();
      }
      (void)hipFree(dA);
      (void)hipFree(dx);
      (void)hipStreamDestroy(s);
    } else {
    int algo = backend == cli::HIP_BLOCKED ? GELIM_GPU_BLOCKED : GELIM_GPU_PIVOT;
    // the blocked LU takes any order up to gelim_gpu_leaf_max_rows() (262144,
    // beyond one GPU's 288 GB at fp64): no silent fallback to hip-pivot
    gelim_gauss_plan* plan = gelim_gauss_plan_create(n, algo, GELIM_PIVOT_PARTIAL, 8, use_graph);
    if (!plan) cli::die("plan_create");
    double *dA = nullptr, *dx = nullptr;
    CLI_HIP(hipMalloc((void**)&dA, A.size() * sizeof(double)));
    CLI_HIP(hipMalloc((void**)&dx, n * sizeof(double)));
    CLI_HIP(hipMemcpy(dA, A.data(), A.size() * sizeof(double), hipMemcpyHostToDevice));
    hipStream_t s;
    CLI_HIP(hipStreamCreate(&s));
    auto run = [&]() {
      CLI_CHECK(gelim_gauss_plan_solve(plan, dA, lda, dx, nullptr, s));
      CLI_HIP(hipStreamSynchronize(s));
    };
    for (int w = 0; w < warmup; ++w) run();
    const double t0 = cli::wall();
    run();
    elapsed = cli::wall() - t0;
    // > 0: 1 + the first zero-pivot column; < 0: a GPU error, not "singular"
    const int info = gelim_gauss_plan_info(plan, s);
    if (info > 0) {
      fprintf(stderr, "The matrix is singular\n");
      exit(-1);
    }
    if (info < 0) cli::die("plan_info");
    CLI_HIP(hipMemcpy(X.data(), dx, n * sizeof(double), hipMemcpyDeviceToHost));
    printf("Device: %s ; Backend: %s ; dtype: f64\n", cli::device_name().c_str(),
           cli::backend_name(backend));
    gelim_gauss_plan_destroy(plan);
    (void)hipFree(dA);
    (void)hipFree(dx);
    (void)hipStreamDestroy(s);
    }
  }

  fprintf(stdout, "Time:  %f seconds\n", elapsed);
  const double error = gelim_error_metric(X.data(), n);
  fprintf(stdout, "Error: %e\n", error);
  if (json)
    printf("{\"program\": \"gauss_external_input\", \"file\": \"%s\", \"n\": %lld, "
           "\"backend\": \"%s\", \"threads\": %s, \"gpus\": %d, \"dtype\": \"f64\", \"time_s\": %.9f, "
           "\"error\": %.6e}\n",
           fname, (long long)n, cli::backend_name(backend),
           cli::is_gpu(backend) ? "null" : std::to_string(num_threads).c_str(), cli::is_gpu(backend) ? 1 : 0,
           elapsed, error);
  return 0;
}
