// Shared helpers for the MEPOL gfx950 kernels (wave64, CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstddef>

#include "../../include/mepol_amd.h"

namespace mepol {

constexpr int kWave = 64;

// Thread-local last-error text behind mepol_last_error_string() (capi.hip).
void set_error(const char* fmt, ...);

#define MEPOL_CHECK_LAUNCH()                                                        \
  do {                                                                              \
    hipError_t e_ = hipGetLastError();                                              \
    if (e_ != hipSuccess) {                                                         \
      ::mepol::set_error("%s:%d: kernel launch failed: %s", __FILE__, __LINE__,     \
                         hipGetErrorString(e_));                                    \
      return (int)e_;                                                               \
    }                                                                               \
  } while (0)

#define MEPOL_HIP(call)                                                             \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      ::mepol::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #call,         \
                         hipGetErrorString(e_));                                    \
      return (int)e_;                                                               \
    }                                                                               \
  } while (0)

// Error codes returned by the C ABI besides hipError_t values.
enum : int {
  kErrBadArg = 1001,
  kErrWorkspace = 1002,
  kErrUnsupported = 1003,
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

__device__ __forceinline__ double shfl_xor_d(double v, int m) { return __shfl_xor(v, m, kWave); }

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, kWave);
  return v;
}

__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, kWave));
  return v;
}

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

}  // namespace mepol
