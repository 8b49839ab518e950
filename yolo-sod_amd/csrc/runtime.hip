// Library-wide runtime pieces of the C ABI: error reporting and version query.
#include "common.h"
#include <string.h>

namespace ys {
static thread_local char g_err[1024] = {0};
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace ys

YS_EXPORT const char* yolosod_last_error(void) { return ys::g_err; }
YS_EXPORT int yolosod_abi_version(void) { return 1; }
