// matrix_gen <matrixorder> — writes the synthetic 2*min(row,col) system in
// the reference `.dat` format to stdout, byte-compatible with
// Pthreads/Version-1/matrices_dense/matrix_gen.cc.
#include <cstdio>
#include <cstdlib>

#include "gelim/gelim.h"

int main(int argc, char* argv[]) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s <matrixorder>\n", argv[0]);
    exit(-1);
  }
  if (gelim_matrix_gen(atoll(argv[1]), "-") != 0) {
    fprintf(stderr, "%s\n", gelim_last_error());
    exit(-1);
  }
  return 0;
}
