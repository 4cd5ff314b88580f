// Diagnostic build (not part of the product ABI): the multi-workgroup rollout kernel of
// mepol_amd/csrc/envs.hip instantiated with PROBE = true, so lane 0 of every workgroup records
// s_memtime spans of the step's phases.  Built by tools/variants/build_rollout_probe.sh, driven
// by tools/rollout_probe.py.
#include <cstdarg>
#include <cstdio>

#include "../../mepol_amd/csrc/envs.hip"

namespace mepol {
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
}
}  // namespace mepol

extern "C" int probe_rollout_mw_gridworld(const double* W1, const double* b1, int h0,
                                          const double* W2t, const double* b2, int h1,
                                          const double* Wm, const double* bm,
                                          const double* log_std, const float* init32,
                                          const double* noise, int64_t n, int64_t T,
                                          float* states_rec, float* actions_rec,
                                          unsigned long long* mail, int* err, long long* probe,
                                          void* stream) {
  const int np = (h1 + 63) / 64, nw = ((h0 > h1 ? h0 : h1) + 63) / 64;
  if (h0 > 306 || h1 > 512) return 1;
  hipFuncSetAttribute((const void*)rollout_mlp_mw_kernel<1, true>,
                      hipFuncAttributeMaxDynamicSharedMemorySize, 306 * 64 * 8);
  hipLaunchKernelGGL((rollout_mlp_mw_kernel<1, true>), dim3((unsigned)(n * np)), dim3(64 * kRollMwWaves),
                     (size_t)h0 * 64 * 8, (hipStream_t)stream, W1, b1, h0, W2t, b2, h1, Wm, bm,
                     log_std, 2, nullptr, init32, noise, n, T, states_rec, actions_rec, nullptr,
                     nullptr, np, nw, mail, err, err + 1, probe);  // err[1]: ticket (zeroed)
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
