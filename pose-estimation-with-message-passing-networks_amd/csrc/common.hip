// Library-level entry points: ABI version, thread-local error string, device check.
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>

#include "pemp_common.h"

namespace pemp {
static thread_local char g_err[512] = "";

bool debug_sync() {
  static const bool on = [] {
    const char* v = getenv("PEMP_DEBUG_SYNC");
    return v && v[0] && v[0] != '0';
  }();
  return on;
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace pemp

extern "C" int pemp_abi_version(void) { return PEMP_ABI_VERSION; }

extern "C" const char* pemp_last_error(void) { return pemp::g_err; }

extern "C" int pemp_device_check(void) {
  int dev = 0;
  PEMP_HIP(hipGetDevice(&dev));
  hipDeviceProp_t prop;
  PEMP_HIP(hipGetDeviceProperties(&prop, dev));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    pemp::set_error("device %d is %s, libpemp is built for gfx950 (MI355X)", dev, prop.gcnArchName);
    return PEMP_ERR_UNSUPPORTED;
  }
  return PEMP_OK;
}
