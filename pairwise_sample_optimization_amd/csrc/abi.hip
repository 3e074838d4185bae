// Error plumbing for the C-ABI: thread-local last-error string, no exceptions cross the boundary.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "common.h"

static thread_local char g_last_error[1024] = "";
static thread_local char g_last_kernel[160] = "";

void pso_note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_kernel, sizeof(g_last_kernel), fmt, ap);
  va_end(ap);
}

void pso_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int pso_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    pso_set_error("%s: %s", what, hipGetErrorString(e));
    return PSO_ERR_HIP;
  }
  return PSO_OK;
}

extern "C" {
const char* pso_last_error(void) { return g_last_error; }
const char* pso_last_kernel(void) { return g_last_kernel; }
int pso_abi_version(void) { return PSO_ABI_VERSION; }
}
