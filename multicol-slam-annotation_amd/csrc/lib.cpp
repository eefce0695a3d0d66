// Library-wide helpers: error text, version, device probing.
#include "common.hpp"
#include <cstdio>
#include <cstring>

namespace mcs {

static thread_local char g_err[512] = "";

void set_error(const char* msg) {
  std::snprintf(g_err, sizeof(g_err), "%s", msg);
}

void set_hip_error(hipError_t e, const char* expr, const char* file, int line) {
  std::snprintf(g_err, sizeof(g_err), "HIP error %d (%s) at %s:%d: %s", (int)e,
                hipGetErrorString(e), file, line, expr);
}

}  // namespace mcs

extern "C" {

const char* mcs_version(void) { return "mcs_amd 0.1.0 (gfx950)"; }

const char* mcs_last_error(void) { return mcs::g_err; }

int32_t mcs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
