// Shared helpers of the libdvh C-ABI: export macro and the thread-local last-error string.
#pragma once
#include <stdint.h>

#define DVH_API extern "C" __attribute__((visibility("default")))

namespace dvh {
// Records `msg` as the calling thread's last error and returns `code` (negative).
int set_error(int code, const char* msg);
// Compute units of the current device (cached on first use; 256 if the query fails).
int cu_count();
}  // namespace dvh
