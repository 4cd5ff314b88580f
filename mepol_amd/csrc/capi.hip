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

extern "C" int mepol_abi_version(void) { return MEPOL_ABI_VERSION; }

// Stream-ordered copy between device and (pinned) host buffers; under stream capture it becomes
// a memcpy node, so a replayed graph can read its scalar inputs from and write its control
// outputs to pinned host memory without separate launches around the replay.
extern "C" int mepol_memcpy_async(void* dst, const void* src, size_t bytes, void* stream) {
  if (!dst || !src) {
    mepol::set_error("mepol_memcpy_async: null pointer");
    return mepol::kErrBadArg;
  }
  if (bytes == 0) return 0;
  MEPOL_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, (hipStream_t)stream));
  return 0;
}
