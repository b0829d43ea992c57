// Host-only sanitizer driver: exercises every CPU
// backend and CPU building block of libgelim's host code so that it can be
// built with -fsanitize=address,undefined or -fsanitize=thread and run
// without a GPU.  The reference's Pthreads V3 has a stack overflow at
// -t > 32 (ASan: dynamic-stack-buffer-overflow) and a racy condvar barrier
// (TSan); this run covers both configurations of ours (40 threads, pinned).
//
//   sanitize_check [mode] [file.dat]    mode: all | pthreads (TSan: no OpenMP)
// Exit 0 when every backend agrees with the sequential reference.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "gelim/gelim.h"

namespace {

int failures = 0;

void expect(bool ok, const std::string& what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what.c_str());
    ++failures;
  }
}

struct System {
  int64_t n;
  std::vector<double> A, b;
};

System random_system(int64_t n, uint64_t seed) {
  System s{n, std::vector<double>(n * n), std::vector<double>(n)};
  gelim_init_random_f64(s.A.data(), n, n, seed);
  gelim_init_rhs_f64(s.A.data(), n, s.b.data(), n);
  return s;
}

std::vector<double> solve_cpu(System s, int backend, int threads, int pivot, int affinity) {
  const int rc = gelim_cpu_gauss(s.A.data(), s.n, s.b.data(), s.n, pivot, backend, threads, affinity);
  expect(rc == GELIM_OK, "gelim_cpu_gauss backend " + std::to_string(backend) + ": " + gelim_last_error());
  std::vector<double> x(s.n);
  gelim_cpu_backsub_unit(s.A.data(), s.n, s.b.data(), x.data(), s.n);
  return x;
}

double max_diff(const std::vector<double>& a, const std::vector<double>& b) {
  double d = 0;
  for (size_t i = 0; i < a.size(); ++i) d = std::fmax(d, std::fabs(a[i] - b[i]));
  return d;
}

void check_backends(bool with_omp) {
  const System s = random_system(97, 5);
  const auto ref = solve_cpu(s, GELIM_CPU_SEQ, 1, GELIM_PIVOT_PARTIAL, 0);
  expect(gelim_error_metric(ref.data(), s.n) < 1e-10, "seq error metric");
  struct Case { int backend, threads, affinity; };
  std::vector<Case> cases = {{GELIM_CPU_PTH_V1, 4, 0}, {GELIM_CPU_PTH_V2, 3, 0}, {GELIM_CPU_PTH_V3, 4, 1},
                             {GELIM_CPU_PTH_V3, 40, 1}};  // > 32: the reference's V3 overflows here
  if (with_omp) cases.push_back({GELIM_CPU_OMP, 4, 0});
  for (const Case& c : cases) {
    const auto x = solve_cpu(s, c.backend, c.threads, GELIM_PIVOT_PARTIAL, c.affinity);
    expect(max_diff(x, ref) == 0.0, "backend " + std::to_string(c.backend) + " x" + std::to_string(c.threads) +
                                        " differs from seq");
  }
  // synthetic internal system, zero-pivot rule: exact (-0.5, 0, ..., 0, 0.5)
  System syn{64, std::vector<double>(64 * 64), std::vector<double>(64)};
  gelim_init_synthetic_f64(syn.A.data(), 64, syn.b.data(), 64);
  const auto xs = solve_cpu(syn, GELIM_CPU_PTH_V3, 8, GELIM_PIVOT_ZERO, 0);
  expect(xs[0] == -0.5 && xs[63] == 0.5 && xs[31] == 0.0, "synthetic exact solution");
}

void check_blocks() {
  const int64_t m = 40, w = 8, nc = 12;
  std::vector<double> P(m * (w + nc));
  gelim_init_random_block_f64(P.data(), w + nc, 0, m, 0, w + nc, 9);
  std::vector<int32_t> piv(w);
  int32_t info = 0;
  expect(gelim_cpu_panel_factor(P.data(), w + nc, m, w, 0, GELIM_PIVOT_PARTIAL, piv.data(), &info) == GELIM_OK,
         "panel_factor");
  expect(gelim_cpu_swap_trsm(P.data() + w, w + nc, nc, P.data(), w + nc, w, piv.data(), 0, m) == GELIM_OK,
         "swap_trsm");
  expect(gelim_cpu_gemm_update(P.data() + w * (w + nc) + w, w + nc, P.data() + w * (w + nc), w + nc, P.data() + w,
                               w + nc, m - w, nc, w) == GELIM_OK,
         "gemm_update");
  for (double v : P) expect(std::isfinite(v), "finite block results");
}

void check_matmul(bool with_omp) {
  const int64_t n = 33;
  std::vector<float> A(n * n), B(n * n), C(n * n), C2(n * n);
  gelim_init_matmul_f32(A.data(), B.data(), n);
  gelim_cpu_matmul_f32(A.data(), B.data(), C.data(), n, 0, 1);
  if (with_omp) {
    gelim_cpu_matmul_f32(A.data(), B.data(), C2.data(), n, 1, 4);
    expect(std::memcmp(C.data(), C2.data(), sizeof(float) * n * n) == 0, "omp matmul == seq matmul");
  }
}

void check_io(const char* path) {
  const int64_t n = gelim_dat_size(path);
  expect(n > 0, std::string("dat_size ") + path);
  if (n <= 0) return;
  std::vector<double> A(n * n);
  expect(gelim_dat_read(path, A.data(), n, n) == GELIM_OK, "dat_read");
  expect(gelim_dat_size("/nonexistent/file.dat") < 0, "missing file reported");
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "all";
  const bool with_omp = mode != "pthreads";
  check_backends(with_omp);
  if (with_omp) check_blocks();  // OpenMP parallel-for: libgomp is not TSan-instrumented
  check_matmul(with_omp);
  if (argc > 2) check_io(argv[2]);
  std::printf("sanitize_check %s: %s\n", mode.c_str(), failures ? "FAILED" : "ok");
  return failures ? 1 : 0;
}
