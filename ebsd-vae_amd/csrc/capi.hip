// Error plumbing and version of the C ABI (include/ebsdvae.h).
#include <stdarg.h>
#include <stdio.h>

#include "common.h"
#include "../../include/ebsdvae.h"

namespace {
thread_local char g_err[512] = "";
}

namespace evh {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return 2;
  }
  return 0;
}
}  // namespace evh

extern "C" const char* ebsdvae_last_error(void) { return g_err; }
extern "C" int ebsdvae_version(void) { return 1; }
