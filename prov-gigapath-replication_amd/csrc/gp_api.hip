// Library-level entry points: version and per-thread error reporting.
#include <stdarg.h>
#include <stdio.h>

#include "gp_api.h"

static thread_local char g_err[512] = "";

void gp_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void gp_clear_error() { g_err[0] = 0; }

int gp_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    gp_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return 0;
}

// GP_ABI_VERSION_OVERRIDE: a lab build whose entry points predate the current header (tools/attn_lab
// liblab_r01.so: the round-1 sources, ABI 4) reports its own version, so the ctypes binding refuses it
#ifdef GP_ABI_VERSION_OVERRIDE
extern "C" int gp_abi_version(void) { return GP_ABI_VERSION_OVERRIDE; }
#else
extern "C" int gp_abi_version(void) { return GP_ABI_VERSION; }
#endif

extern "C" const char* gp_last_error_string(void) { return g_err; }
