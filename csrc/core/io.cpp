// L1 data / IO: the reference `.dat` coordinate format and the matrix_gen
// generator.
//
// Reference behaviour:
//   header  "n n nnz"  (only the first field is used; nnz is ignored)
//   entries "row col value", 1-based, until a line whose row field is 0
//   (Pthreads/Version-1/gauss_external_input.c:34-86).
// Differences on purpose: lines of any length, a missing terminator ends the
// file instead of looping on a stale buffer, out-of-range indices are an error
// instead of a heap overwrite, 64-bit sizes.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gelim/internal.h"

namespace {

struct File {
  FILE* f = nullptr;
  explicit File(const char* p, const char* mode) : f(std::fopen(p, mode)) {}
  ~File() {
    if (f && f != stdout) std::fclose(f);
  }
};

// Read one line into `buf` (grown as needed). Returns false at EOF.
bool read_line(FILE* f, std::string& buf) {
  buf.clear();
  char chunk[4096];
  while (std::fgets(chunk, sizeof chunk, f)) {
    buf += chunk;
    if (!buf.empty() && buf.back() == '\n') return true;
  }
  return !buf.empty();
}

}  // namespace

extern "C" int64_t gelim_dat_size(const char* path) {
  File fh(path, "r");
  if (!fh.f) return GELIM_FAIL(GELIM_E_IO, "The matrix file open error");
  std::string line;
  if (!read_line(fh.f, line))
    return GELIM_FAIL(GELIM_E_IO, std::string("empty matrix file: ") + path);
  long long l1 = 0;
  if (std::sscanf(line.c_str(), "%lld", &l1) != 1 || l1 <= 0)
    return GELIM_FAIL(GELIM_E_IO, std::string("bad header in ") + path);
  return (int64_t)l1;
}

extern "C" int gelim_dat_read(const char* path, double* out, int64_t n,
                              int64_t ld) {
  if (!out || n <= 0 || ld < n) return GELIM_FAIL(GELIM_E_ARG, "bad dat_read args");
  File fh(path, "r");
  if (!fh.f) return GELIM_FAIL(GELIM_E_IO, "The matrix file open error");
  std::string line;
  read_line(fh.f, line);  // header (validated by gelim_dat_size)
  for (int64_t i = 0; i < n; ++i) std::memset(out + i * ld, 0, sizeof(double) * n);
  int64_t lineno = 1;
  while (read_line(fh.f, line)) {
    ++lineno;
    char* p = const_cast<char*>(line.c_str());
    char* e = nullptr;
    long long r = std::strtoll(p, &e, 10);
    if (e == p) continue;  // blank line
    if (r == 0) break;     // terminator "0 0 0"
    p = e;
    long long c = std::strtoll(p, &e, 10);
    if (e == p) return GELIM_FAIL(GELIM_E_IO, "bad entry at line " + std::to_string(lineno));
    p = e;
    double v = std::strtod(p, &e);
    if (e == p) return GELIM_FAIL(GELIM_E_IO, "bad value at line " + std::to_string(lineno));
    if (r < 1 || r > n || c < 1 || c > n)
      return GELIM_FAIL(GELIM_E_IO, "index out of range at line " + std::to_string(lineno));
    out[(r - 1) * ld + (c - 1)] = v;
  }
  return GELIM_OK;
}

// Byte-compatible with matrix_gen.cc (GEN:13-22): header "n n n*n", entries
// column-major with value 2*min(row,col) printed "%f", terminator "0 0 0".
extern "C" int gelim_matrix_gen(int64_t n, const char* path) {
  if (n <= 0) return GELIM_FAIL(GELIM_E_ARG, "matrix order must be positive");
  FILE* f = (!path || std::strcmp(path, "-") == 0) ? stdout : std::fopen(path, "w");
  if (!f) return GELIM_FAIL(GELIM_E_IO, std::string("cannot write ") + path);
  std::vector<char> buf(1 << 20);
  if (f != stdout) std::setvbuf(f, buf.data(), _IOFBF, buf.size());
  std::fprintf(f, "%lld %lld %lld\n", (long long)n, (long long)n, (long long)(n * n));
  for (int64_t col = 1; col <= n; ++col)
    for (int64_t row = 1; row <= n; ++row) {
      double value = (row < col) ? 2.0 * row : 2.0 * col;
      std::fprintf(f, "%lld %lld %f\n", (long long)row, (long long)col, value);
    }
  std::fprintf(f, "0 0 0\n");
  std::fflush(f);
  if (f != stdout) std::fclose(f);
  return GELIM_OK;
}
