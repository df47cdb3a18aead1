// Library-level entry points of libllp_hip.so: version, errors, device probe.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>

#include "../../include/llp_hip.h"

namespace llp {
thread_local char g_err[512] = "";
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
thread_local const char* g_kernel = "";
void note_kernel(const char* name) { g_kernel = name; }
}  // namespace llp

extern "C" int llp_version(void) { return 1; }

extern "C" const char* llp_last_error(void) { return llp::g_err; }

extern "C" const char* llp_last_gemm_kernel(void) { return llp::g_kernel; }

extern "C" int llp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
