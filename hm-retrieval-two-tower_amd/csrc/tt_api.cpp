// Version string and thread-local error reporting for the libtt C ABI.
#include <cstdio>
#include <cstring>

#include "tt_common.h"

namespace tt {

static thread_local char g_last_error[1024] = {0};

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { g_last_error[0] = 0; }

}  // namespace tt

extern "C" const char* tt_version(void) { return "tt 0.1.0 gfx950"; }

extern "C" const char* tt_last_error(void) { return tt::g_last_error; }
