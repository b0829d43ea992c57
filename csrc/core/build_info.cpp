// Build provenance: the digest of the sources this libgelim.so was compiled
// from (csrc/cmake/source_digest.cmake), so a shipped library can be checked
// against the tree beside it (gelim._native.source_digest,
// tests/test_build_provenance.py).
#include "gelim_digest.h"

extern "C" const char* gelim_build_digest(void) { return GELIM_SOURCE_DIGEST; }
