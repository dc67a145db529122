// srpde-mi355x C-ABI housekeeping: thread-local error text and version.
#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace srpde {

static thread_local char g_err[512] = "";
static thread_local char g_kern[192] = "";

void note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kern, sizeof(g_kern), fmt, ap);
  va_end(ap);
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

}  // namespace srpde

extern "C" {

const char* srpde_last_error(void) { return srpde::g_err; }

const char* srpde_last_kernel(void) { return srpde::g_kern; }

int srpde_version(void) { return SRPDE_ABI_VERSION; }

}  // extern "C"
