// Error plumbing and identification for libhiseg.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include "hiseg.h"

static thread_local char g_err[512] = "";

void hiseg_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hiseg_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    hiseg_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return HISEG_ERR_LAUNCH;
  }
  return HISEG_OK;
}

extern "C" int hiseg_version(void) { return 100; }
extern "C" const char* hiseg_last_error_string(void) { return g_err; }
extern "C" int hiseg_built_for_gfx950(void) { return 1; }
