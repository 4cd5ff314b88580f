// Scalar traffic between the host and a replayed iteration graph (algorithms/device_loop.py)
// without memcpy nodes: the per-replay inputs (enable flag, learning rate, bias corrections)
// and the two control outputs (H, KL) live in pinned host memory mapped into the device address
// space, and one-wave kernels move them.  A memcpy node costs a DMA hand-off on each side of the
// copy (the round-2 iteration timeline: ~45 us of copies and gaps per iteration around three
// 16-64-byte copies and a concatenation); a kernel node is ordered like every other launch.
#include "common.hpp"

namespace mepol {
namespace hostio {

// Accesses to the mapped host words are system-scope atomics (sc0 sc1: no GPU cache keeps a
// stale copy between replays; the host rewrites the inputs before every launch).
__device__ __forceinline__ double sys_load(const double* p) {
  return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const long long*>(p),
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ void sys_store(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// mode 0: dst (device) <- src (mapped host); mode 1: dst (mapped host) <- src (device)
__global__ void small_copy_kernel(double* dst, const double* src, int n, int mode) {
  const int i = threadIdx.x;
  if (i >= n) return;
  if (mode == 0)
    dst[i] = sys_load(src + i);
  else
    sys_store(dst + i, src[i]);
}

// vals[0] = a[ia], vals[1] = b[ib] (read first), then cur[0..n) = nw[0..n): the iteration's
// (H(theta_t), KL(theta_t+1)) out and the entropy sums of theta_t+1 kept for the next replay.
__global__ void scalars_emit_kernel(const double* a, int ia, const double* b, int ib,
                                    double* vals, double* cur, const double* nw, int n) {
  if (threadIdx.x != 0) return;
  const double va = a[ia], vb = b[ib];
  for (int i = 0; i < n; ++i) cur[i] = nw[i];
  sys_store(vals, va);
  sys_store(vals + 1, vb);
}

}  // namespace hostio
}  // namespace mepol

using namespace mepol;

extern "C" int mepol_host_alloc_mapped(size_t bytes, void** host_ptr, void** dev_ptr) {
  if (!host_ptr || !dev_ptr || bytes == 0) {
    set_error("mepol_host_alloc_mapped: bad arguments");
    return kErrBadArg;
  }
  void* h = nullptr;
  // coherent (fine-grained): device accesses are never served from a GPU cache
  MEPOL_HIP(hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  void* d = nullptr;
  hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    set_error("mepol_host_alloc_mapped: hipHostGetDevicePointer failed: %s", hipGetErrorString(e));
    return (int)e;
  }
  *host_ptr = h;
  *dev_ptr = d;
  return 0;
}

extern "C" int mepol_host_free(void* host_ptr) {
  if (host_ptr) MEPOL_HIP(hipHostFree(host_ptr));
  return 0;
}

extern "C" int mepol_small_copy(double* dst, const double* src, int n, int to_host,
                                void* stream) {
  if (!dst || !src || n < 0 || n > 64) {
    set_error("mepol_small_copy: bad arguments (n <= 64)");
    return kErrBadArg;
  }
  if (n == 0) return 0;
  hipLaunchKernelGGL(hostio::small_copy_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst,
                     src, n, to_host ? 1 : 0);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_scalars_emit(const double* a, int ia, const double* b, int ib, double* vals,
                                  double* cur, const double* nw, int n, void* stream) {
  if (!a || !b || !vals || (n > 0 && (!cur || !nw)) || n < 0 || n > 64) {
    set_error("mepol_scalars_emit: bad arguments");
    return kErrBadArg;
  }
  hipLaunchKernelGGL(hostio::scalars_emit_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a,
                     ia, b, ib, vals, cur, nw, n);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
