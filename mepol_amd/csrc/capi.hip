// C-ABI plumbing shared by every entry point: error text, version, device query.
#include "common.hpp"

#include <cstdarg>
#include <cstdio>

namespace mepol {
static thread_local char g_err[1024] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace mepol

extern "C" const char* mepol_last_error_string(void) { return mepol::g_err; }

extern "C" int mepol_abi_version(void) { return 1; }
