// libdvh C-ABI common entry points: version and last-error reporting (include/dvh.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "dvh_common.h"
#include "dvh.h"

namespace dvh {
static thread_local char g_err[256] = "";

int set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg ? msg : "unknown error");
  return code;
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess)
      n = v;
    if (n <= 0) n = 256;
  }
  return n;
}
}  // namespace dvh

DVH_API const char* dvh_last_error(void) { return dvh::g_err; }

DVH_API int dvh_abi_version(void) { return 2; }  // 2: device tables, validated stacking, raw ridge picks
