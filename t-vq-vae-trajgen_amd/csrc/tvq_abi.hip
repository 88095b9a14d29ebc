// ABI plumbing: thread-local error string and version.
#include <stdarg.h>
#include <stdio.h>

#include "tvq_common.h"

namespace tvq {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace tvq

extern "C" const char* tvq_last_error(void) { return tvq::g_err; }
extern "C" int tvq_abi_version(void) { return 1; }
