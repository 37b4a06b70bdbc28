// Error plumbing and version info of libsvla.so (thread-local last-error string).
#include <stdarg.h>

#include "svla_common.h"

namespace svla {
static thread_local char g_err[1024] = "";

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
    return SVLA_ERR_HIP;
  }
  return SVLA_OK;
}

// compute units of the current device (cached per device; 256 on MI355X)
int num_cus() {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    cus[dev] = v;
  }
  return cus[dev];
}
}  // namespace svla

extern "C" const char* svla_last_error(void) { return svla::g_err; }

extern "C" const char* svla_version(void) { return "svla 0.1 gfx950 (CDNA4) bf16-MFMA"; }
