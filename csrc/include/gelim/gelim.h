/*
 * gelim — MI355X-native dense Gaussian elimination and matrix multiply.
 *
 * Public C ABI of libgelim.so.  Everything the Python package, the CLIs and
 * the distributed drivers call goes through this header; the library itself
 * is C++17 (host) + HIP for gfx950 (device).
 *
 * Conventions
 *   - Matrices are ROW-MAJOR with an explicit leading dimension (elements),
 *     matching the reference's contiguous `double **matrix` table
 *     (Pthreads/Version-1/gauss_internal_input.c:29-52).
 *   - All sizes/indices are int64_t (the reference's `int n*n` overflows at
 *     n >= 46341).
 *   - Functions return 0 on success, a negative GELIM_E* code on failure;
 *     gelim_last_error() gives a human-readable message (thread-local).
 *   - `stream` arguments are hipStream_t passed as void* (0 = default
 *     stream) so Python can hand over torch.cuda.current_stream().cuda_stream.
 *   - Device pointers are hipMalloc'ed (or torch CUDA tensor storage).
 */
#ifndef GELIM_GELIM_H
#define GELIM_GELIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ------------------------------------------------------- */
#define GELIM_OK 0
#define GELIM_E_ARG -1      /* bad argument */
#define GELIM_E_IO -2       /* file open / parse error */
#define GELIM_E_HIP -3      /* HIP runtime error */
#define GELIM_E_SINGULAR -4 /* zero pivot encountered */
#define GELIM_E_NOMEM -5    /* allocation failure */
#define GELIM_E_THREAD -6   /* pthread_create failure */

const char* gelim_last_error(void);
const char* gelim_version(void);

/* ---- enums -------------------------------------------------------------- */
/* Pivoting rule.
 *  ZERO    : swap only if A[i][i]==0, taking the first non-zero row below
 *            (reference "internal" getPivot, gauss_internal_input.c:75-121).
 *  PARTIAL : argmax |A[r][i]| for r>=i, ties -> lowest row
 *            (reference "external" getPivot, gauss_external_input.c:125-150). */
enum { GELIM_PIVOT_ZERO = 0, GELIM_PIVOT_PARTIAL = 1 };

/* CPU backends. */
enum {
  GELIM_CPU_SEQ = 0,    /* single thread, reference loop order            */
  GELIM_CPU_OMP = 1,    /* OpenMP parallel-for over rows (S4)             */
  GELIM_CPU_PTH_V1 = 2, /* pthreads fork-join row-cyclic per pivot (S1)   */
  GELIM_CPU_PTH_V2 = 3, /* pthreads column-blocked row-cyclic (S2)        */
  GELIM_CPU_PTH_V3 = 4  /* persistent pthreads + barrier + affinity (S3)  */
};

/* GPU Gauss algorithms. */
enum {
  GELIM_GPU_BLOCKED = 0, /* right-looking blocked LU, fp64 MFMA trailing GEMM   */
  GELIM_GPU_PIVOT = 1    /* reference per-pivot algorithm, one step per column */
};

/* GPU fp32 matmul kernels (SURVEY.md §2.4 K1/K2/K3'). */
enum {
  GELIM_MM_NAIVE_ROW = 0,  /* K1: one workgroup per output row             */
  GELIM_MM_NAIVE_ELEM = 1, /* K2: one thread per output element, 2-D grid   */
  GELIM_MM_MFMA = 2        /* K3': LDS-tiled v_mfma_f32_32x32x2_f32 GEMM    */
};

/* ---- data / IO (L1) ----------------------------------------------------- */
/* Read the header of a reference `.dat` coordinate file; returns n (>0) or a
 * negative error code.  Format: "n n nnz" then "row col value" (1-based)
 * terminated by a row==0 line (gauss_external_input.c:34-86). */
int64_t gelim_dat_size(const char* path);
/* Densify a `.dat` file into `out` (n x n, row-major, leading dim ld). */
int gelim_dat_read(const char* path, double* out, int64_t n, int64_t ld);
/* Write matrix_gen-compatible text for order n to `path` ("-" = stdout). */
int gelim_matrix_gen(int64_t n, const char* path);

/* Synthetic "internal" system: A[i][j] = 2*min(i+1,j+1), b[i] = i. */
void gelim_init_synthetic_f64(double* A, int64_t lda, double* b, int64_t n);
/* Random system: A[i][j] ~ U[-1,1) from a counter-based hash of (seed,i,j). */
void gelim_init_random_f64(double* A, int64_t lda, int64_t n, uint64_t seed);
/* Block of the random matrix: out[r][c] = A[row0+r][col0+c] (same values as
 * gelim_init_random_f64 of the full matrix). */
void gelim_init_random_block_f64(double* out, int64_t ld, int64_t row0, int64_t nrows,
                                 int64_t col0, int64_t ncols, uint64_t seed);
/* R = A * X__ with X__[i] = i+1 (gauss_external_input.c:90-108). */
void gelim_init_rhs_f64(const double* A, int64_t lda, double* R, int64_t n);
/* max_i |x_i - (i+1)| / (i+1)  (gauss_external_input.c:308-315). */
double gelim_error_metric(const double* x, int64_t n);

/* ---- CPU reference backends (L2/L3) ------------------------------------- */
/* Forward elimination in place, reference semantics: A becomes unit upper
 * triangular with zeros below, b is transformed.  threads<=0 -> default.
 * affinity: V3 only (pin thread t to CPU t when threads <= nprocs). */
int gelim_cpu_gauss(double* A, int64_t lda, double* b, int64_t n, int pivot,
                    int backend, int threads, int affinity);
/* Threads an OpenMP region would use (omp_get_max_threads). */
int gelim_cpu_max_threads(void);
/* Back substitution on a unit upper triangle, j descending
 * (gauss_internal_input.c:212-227). */
void gelim_cpu_backsub_unit(const double* U, int64_t ldu, const double* b,
                            double* x, int64_t n);
/* fp32 matmul, exact reference i-j-k loop order (cuda_matmul.cu:28-57). */
void gelim_cpu_matmul_f32(const float* A, const float* B, float* C,
                          int64_t n, int omp, int threads);
/* Reference matmul initialiser: A[idx]=idx+1, B[idx]=1/(idx+1)
 * (cuda_matmul.cu:121-132, with exact integer indices). */
void gelim_init_matmul_f32(float* A, float* B, int64_t n);

/* CPU building blocks of the blocked LU (used by the distributed driver on
 * CPU/gloo and as GPU test oracles). Same contracts as the gelim_gpu_* ones. */
int gelim_cpu_panel_factor(double* P, int64_t ldp, int64_t m, int64_t w,
                           int64_t row0, int pivot, int32_t* piv, int32_t* info);
int gelim_cpu_swap_trsm(double* C, int64_t ldc, int64_t ncols,
                        const double* L, int64_t ldl, int64_t w,
                        const int32_t* piv, int64_t row0, int64_t nrows);
int gelim_cpu_gemm_update(double* C, int64_t ldc, const double* L, int64_t ldl,
                          const double* U, int64_t ldu, int64_t M, int64_t N,
                          int64_t K);

/* ---- GPU runtime ------------------------------------------------------- */
int gelim_gpu_device_count(void);
int gelim_gpu_set_device(int dev);
int gelim_gpu_sync(void* stream);
void* gelim_gpu_malloc(int64_t bytes);
int gelim_gpu_free(void* p);
int gelim_gpu_memcpy_h2d(void* dst, const void* src, int64_t bytes, void* stream);
int gelim_gpu_memcpy_d2h(void* dst, const void* src, int64_t bytes, void* stream);

/* Device initialisers (augmented layout: column n of A holds b). */
int gelim_gpu_init_synthetic(double* dA, int64_t lda, int64_t n, void* stream);
int gelim_gpu_init_synthetic_f32(float* dA, int64_t lda, int64_t n, void* stream);
int gelim_gpu_init_random(double* dA, int64_t lda, int64_t n, uint64_t seed,
                          void* stream);
int gelim_gpu_init_random_block(double* dA, int64_t lda, int64_t row0, int64_t nrows,
                                int64_t col0, int64_t ncols, uint64_t seed, void* stream);
/* dA[:, n] = dA[:, :n] @ (1..n)  (device initRHS). */
int gelim_gpu_init_rhs(double* dA, int64_t lda, int64_t n, void* stream);
/* Max relative error vs (i+1) written to *d_err (device double). */
int gelim_gpu_error_metric(const double* dx, int64_t n, double* d_err,
                           void* stream);

/* ---- GPU building blocks of the blocked LU -------------------------------
 * Panel: factor P (m x w, row-major, ldp) with the given pivot rule;
 * piv[j] receives the LOCAL row (0..m-1) swapped into position j, rows are
 * physically swapped inside the panel, L (unit, below diag) and U overwrite P.
 * info: if a zero pivot appears at column j and *info==0, *info = row0+j+1.
 * Requires m <= 8192*... (see gelim_gpu_panel_max_rows). */
int gelim_gpu_panel_factor(double* dP, int64_t ldp, int64_t m, int64_t w,
                           int64_t row0, int pivot, int32_t* dpiv,
                           int32_t* dinfo, void* stream);
int64_t gelim_gpu_panel_max_rows(int64_t w);
/* Apply the w sequential swaps piv[] (local rows, as produced by the panel)
 * to C (nrows x ncols, ld ldc, rows relative to the panel's first row), then
 * C[0:w,:] = L11^{-1} C[0:w,:] with L11 = unit-lower part of L (ld ldl). */
int gelim_gpu_swap_trsm(double* dC, int64_t ldc, int64_t ncols,
                        const double* dL, int64_t ldl, int64_t w,
                        const int32_t* dpiv, int64_t nrows, void* stream);
/* C (M x N) -= L (M x K) * U (K x N); fp64 MFMA (v_mfma_f64_16x16x4_f64). */
/* C (M x N, ldc) += alpha * A (M x K, lda) * B (K x N, ldb) on the fp64
 * matrix cores (LDS-tiled v_mfma_f64_16x16x4_f64).  A, B 16-byte aligned,
 * lda / ldb / K even, ldb > N when N is odd. */
int gelim_gpu_dgemm(double* dC, int64_t ldc, const double* dA, int64_t lda, const double* dB,
                    int64_t ldb, int64_t M, int64_t N, int64_t K, double alpha, void* stream);
/* the same as a persistent kernel on at most max_wg CUs (one 512-thread
 * workgroup per CU, two tiles each) -- the lookahead side stream's form */
int gelim_gpu_dgemm_capped(double* dC, int64_t ldc, const double* dA, int64_t lda, const double* dB,
                           int64_t ldb, int64_t M, int64_t N, int64_t K, double alpha, int max_wg, void* stream);
/* Wide-panel LU pieces (biglu.hip), exposed for tests: factor the m x 32
 * leaf at dA (its diagonal is row/column c0 of the system: dipiv[c0 + j]
 * gets the absolute LAPACK pivot row of column c0 + j, dpairs the net row
 * movement relative to c0), and apply a movement (dpairs may be NULL) to
 * columns [0, lend) and [rbeg, rend) of rows [c0, ...) plus the TRSM of the
 * 32 rows from c0 (L11 = the leaf at (c0, c0)) on right columns below
 * trsm_end (dA: row c0, column 0 of the system). */
int gelim_gpu_leaf_factor(double* dA, int64_t lda, int64_t m, int64_t c0, int pivot, int32_t* dipiv,
                          int32_t* dpairs, int32_t* dinfo, void* stream);
int gelim_gpu_laswp_trsm(double* dA, int64_t lda, int64_t c0, int64_t lend, int64_t rbeg, int64_t rend,
                         int64_t trsm_end, int64_t nrows, const int32_t* dpairs, void* stream);
/* U12 = L11^-1 C: nb (<= 256, multiple of 32) rows of C over ncols columns,
 * L11 the unit-lower nb x nb block at dL; max_wg > 0 caps the grid */
int gelim_gpu_panel_trsm(double* dC, int64_t ldc, int64_t ncols, int64_t nb, const double* dL, int64_t ldl,
                         int max_wg, void* stream);
/* a whole outer panel's interchanges (nleaves leaf pair lists, `slot` ints
 * apart, diagonals c0, c0 + 32, ...) on columns [lbeg, lend) and
 * [rbeg, rend) of the n-row system at dA (row 0, column 0); max_wg > 0
 * caps the grid */
int gelim_gpu_laswp_panel(double* dA, int64_t lda, int64_t n, int64_t c0, int nleaves, const int32_t* dpairs,
                          int64_t slot, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, int max_wg,
                          void* stream);
/* the same movement composed into one permutation first (<= 512 moved rows,
 * dnet: 1 + 128 * nleaves ints of device scratch), then gathered/scattered */
int gelim_gpu_laswp_net(double* dA, int64_t lda, int64_t n, int64_t c0, int nleaves, const int32_t* dpairs,
                        int64_t slot, int64_t lbeg, int64_t lend, int64_t rbeg, int64_t rend, int32_t* dnet,
                        int max_wg, void* stream);
int gelim_gpu_gemm_update(double* dC, int64_t ldc, const double* dL,
                          int64_t ldl, const double* dU, int64_t ldu,
                          int64_t M, int64_t N, int64_t K, void* stream);
/* Solve U x = y for upper-triangular U (n x n, ldu). unit!=0: unit diagonal.
 * y is read from dy (stride incy), x written to dx; dbnorm (optional, may be
 * NULL) receives y[i]/U[i][i] (the reference's transformed B). */
int gelim_gpu_backsub(const double* dU, int64_t ldu, const double* dy,
                      int64_t incy, double* dx, double* dbnorm, int64_t n,
                      int unit, void* stream);

/* ---- GPU Gauss solver plan ---------------------------------------------
 * A plan owns a device working copy of the augmented system [A | b]
 * (n x (n+1), padded leading dimension) plus pivot/info workspace, and a
 * captured hipGraph of the whole elimination + back substitution. */
typedef struct gelim_gauss_plan gelim_gauss_plan;

gelim_gauss_plan* gelim_gauss_plan_create(int64_t n, int algo, int pivot,
                                          int dtype_bytes, int use_graph);
void gelim_gauss_plan_destroy(gelim_gauss_plan* p);
int64_t gelim_gauss_plan_lda(const gelim_gauss_plan* p);
/* Device pointer of the plan's working augmented matrix (n x lda). */
void* gelim_gauss_plan_work(gelim_gauss_plan* p);
/* Solve. d_src_aug: optional device augmented matrix (n x (n+1), ld src_ld)
 * copied into the working buffer first (NULL: solve what is already in the
 * working buffer). dx: device solution (n). dbnorm: optional transformed b.
 * The elimination + back substitution are enqueued on `stream`; when the plan
 * uses a graph it is captured on first use per (src, dx, dbnorm) triple. */
int gelim_gauss_plan_solve(gelim_gauss_plan* p, const void* d_src_aug,
                           int64_t src_ld, void* dx, void* dbnorm,
                           void* stream);
/* Reads back the info word (synchronises the stream). 0 = non-singular,
 * k>0: first zero pivot at column k-1. */
int gelim_gauss_plan_info(gelim_gauss_plan* p, void* stream);
/* hip-pivot plans keep their factors: re-solve A x = c (fp64 device vectors)
 * in O(n^2) after a solve */
int gelim_gauss_plan_resolve(gelim_gauss_plan* p, const double* d_c, double* d_x, void* stream);
/* r = b - A x of an augmented fp64 system (b in column n) */
int gelim_gpu_residual(const double* d_aug, int64_t ld, int64_t n, const double* d_x, double* d_r, void* stream);

/* ---- randomised no-pivoting engine (hip-rbt / hip-mixed) ----------------
 * Random butterfly transform + block LDU without pivoting (lu_mixed.hip).
 * ud / vd: host arrays of 2 * gelim_mixed_padded(n) butterfly entries each
 * (exp(r / 10), r uniform in [-1/2, 1/2]); fp64 = 1: fp64 factors (hip-rbt). */
typedef struct gelim_mixed_plan gelim_mixed_plan;
int64_t gelim_mixed_max_n(void);
int64_t gelim_mixed_padded(int64_t n);
gelim_mixed_plan* gelim_mixed_plan_create2(int64_t n, const double* ud, const double* vd, int fp64);
void gelim_mixed_plan_destroy(gelim_mixed_plan* p);
/* Whole solve with fp64 refinement to a componentwise backward error <= 4 eps:
 * 0 = x written, 1 = fall back to partial pivoting, < 0 = error. */
int gelim_mixed_solve(gelim_mixed_plan* p, const double* d_aug, int64_t ld, double* d_x, int max_steps, int* steps,
                      double* berr, void* stream);

/* ---- GPU fp32 matmul --------------------------------------------------- */
/* C (M x N) = A (M x K) * B (K x N), row-major, ld = cols. */
int gelim_gpu_matmul_f32(const float* dA, const float* dB, float* dC,
                         int64_t M, int64_t N, int64_t K, int kernel,
                         void* stream);

/* General form: C = A*B (+ C if accumulate), explicit leading dimensions so
 * column slices of larger row-major matrices can be used directly. */
int gelim_gpu_matmul_f32_ex(const float* dA, int64_t lda, const float* dB, int64_t ldb,
                            float* dC, int64_t ldc, int64_t M, int64_t N, int64_t K,
                            int accumulate, int kernel, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GELIM_GELIM_H */
