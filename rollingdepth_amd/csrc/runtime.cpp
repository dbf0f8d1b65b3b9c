// librdmi runtime: thread-local error reporting and version.
#include "common.h"

#include <string.h>

namespace rdmi {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

}  // namespace rdmi

extern "C" const char* rdmi_last_error(void) { return rdmi::g_err; }
extern "C" int rdmi_version(void) { return 1; }
