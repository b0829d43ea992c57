// Error reporting for the C ABI.
#include <string>

#include "gelim/internal.h"

namespace gelim {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const char* file, int line, const std::string& msg) {
  const char* base = file;
  for (const char* p = file; *p; ++p)
    if (*p == '/') base = p + 1;
  g_last_error = std::string(base) + ":" + std::to_string(line) + ": " + msg;
  return code;
}

}  // namespace gelim

extern "C" const char* gelim_last_error(void) {
  return gelim::g_last_error.c_str();
}

extern "C" const char* gelim_version(void) { return "gelim 0.1.0 (gfx950)"; }
