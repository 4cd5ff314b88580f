// Parameter update of the off-policy loop: torch.optim.Adam / RMSprop with the defaults MEPOL
// uses (src/algorithms/mepol.py:308-311: Adam(lr) or RMSprop(lr); no weight decay, amsgrad,
// momentum or centering), applied to the target policy's tensors in one launch.
//
// Element math follows torch's multi-tensor (foreach) implementation step by step, one IEEE
// rounding per torch op (built with -ffp-contract=off):
//   Adam:    m = m + (1-b1)(g - m)                       _foreach_lerp_ (weight < 0.5 branch)
//            v = v*b2;  v = v + (1-b2)(g*g)              _foreach_mul_, _foreach_addcmul_
//            d = sqrt(v) / bc2_sqrt + eps                _foreach_sqrt, _div_, _add_
//            p = p + (-step_size)(m / d)                 _foreach_addcdiv_
//   RMSprop: v = v*alpha;  v = v + (1-alpha)(g*g);  d = sqrt(v) + eps;  p = p + (-lr)(g / d)
// The per-step scalars come from device memory (scal[]), so a captured graph picks up the
// host-computed bias corrections / learning rate of each replay; scal[0] == 0 disables the
// update (graph warm-up).  Optional snapshot pointers receive p, m, v as they were before the
// update (the device iteration's shadow of theta and its moment snapshot, so a speculative
// replay can be undone without separate copy launches).
#include "common.hpp"

#include <algorithm>

namespace mepol {
namespace optim {

constexpr int kMaxTensors = 8;

struct Tensors {
  double* p[kMaxTensors];
  const double* g[kMaxTensors];
  double* m[kMaxTensors];
  double* v[kMaxTensors];
  int64_t n[kMaxTensors];
  double* ps[kMaxTensors];  // snapshots (nullptr: none)
  double* ms[kMaxTensors];
  double* vs[kMaxTensors];
};

// scal: [enable, step_size, bc2_sqrt, beta1, beta2, eps]
__global__ __launch_bounds__(256) void adam_kernel(Tensors t, const double* __restrict__ scal) {
  if (scal[0] == 0.0) return;
  const int ti = blockIdx.y;
  const int64_t n = t.n[ti];
  double* __restrict__ p = t.p[ti];
  const double* __restrict__ g = t.g[ti];
  double* __restrict__ m = t.m[ti];
  double* __restrict__ v = t.v[ti];
  double* ps = t.ps[ti];
  double* ms = t.ms[ti];
  double* vs = t.vs[ti];
  const double step_size = scal[1], bc2_sqrt = scal[2], b1 = scal[3], b2 = scal[4], eps = scal[5];
  const double w1 = 1.0 - b1, w2 = 1.0 - b2, neg_step = -step_size;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double gi = g[i], m0 = m[i], v0 = v[i], p0 = p[i];
    if (ps) ps[i] = p0;
    if (ms) ms[i] = m0;
    if (vs) vs[i] = v0;
    const double mi = m0 + w1 * (gi - m0);
    const double vi = v0 * b2 + w2 * (gi * gi);
    const double d = sqrt(vi) / bc2_sqrt + eps;
    m[i] = mi;
    v[i] = vi;
    p[i] = p0 + neg_step * (mi / d);
  }
}

// scal: [enable, lr, alpha, eps]
__global__ __launch_bounds__(256) void rmsprop_kernel(Tensors t, const double* __restrict__ scal) {
  if (scal[0] == 0.0) return;
  const int ti = blockIdx.y;
  const int64_t n = t.n[ti];
  double* __restrict__ p = t.p[ti];
  const double* __restrict__ g = t.g[ti];
  double* __restrict__ v = t.v[ti];
  double* ps = t.ps[ti];
  double* vs = t.vs[ti];
  const double neg_lr = -scal[1], alpha = scal[2], eps = scal[3], w = 1.0 - alpha;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double gi = g[i], v0 = v[i], p0 = p[i];
    if (ps) ps[i] = p0;
    if (vs) vs[i] = v0;
    const double vi = v0 * alpha + w * (gi * gi);
    v[i] = vi;
    p[i] = p0 + neg_lr * (gi / (sqrt(vi) + eps));
  }
}

}  // namespace optim
}  // namespace mepol

using namespace mepol;
using namespace mepol::optim;

extern "C" int mepol_optim_step_snapshot(int kind, int n_tensors, double* const* params,
                                         const double* const* grads, double* const* exp_avg,
                                         double* const* exp_avg_sq, const int64_t* sizes,
                                         const double* scalars, double* const* params_snap,
                                         double* const* exp_avg_snap,
                                         double* const* exp_avg_sq_snap, void* stream) {
  if ((kind != 0 && kind != 1) || n_tensors <= 0 || n_tensors > kMaxTensors || !params || !grads ||
      !exp_avg_sq || !sizes || !scalars || (kind == 0 && !exp_avg)) {
    set_error("mepol_optim_step: bad arguments (kind 0=Adam/1=RMSprop, 1..%d tensors)",
              kMaxTensors);
    return kErrBadArg;
  }
  Tensors t{};
  int64_t nmax = 1;
  for (int i = 0; i < n_tensors; ++i) {
    if (!params[i] || !grads[i] || !exp_avg_sq[i] || (kind == 0 && !exp_avg[i]) || sizes[i] < 0) {
      set_error("mepol_optim_step: null tensor %d", i);
      return kErrBadArg;
    }
    t.p[i] = params[i];
    t.g[i] = grads[i];
    t.m[i] = kind == 0 ? exp_avg[i] : nullptr;
    t.v[i] = exp_avg_sq[i];
    t.n[i] = sizes[i];
    t.ps[i] = params_snap ? params_snap[i] : nullptr;
    t.ms[i] = (kind == 0 && exp_avg_snap) ? exp_avg_snap[i] : nullptr;
    t.vs[i] = exp_avg_sq_snap ? exp_avg_sq_snap[i] : nullptr;
    nmax = sizes[i] > nmax ? sizes[i] : nmax;
  }
  const unsigned gx = (unsigned)std::min<int64_t>((nmax + 255) / 256, 1024);
  dim3 grid(gx, n_tensors);
  hipStream_t st = (hipStream_t)stream;
  if (kind == 0)
    hipLaunchKernelGGL(adam_kernel, grid, dim3(256), 0, st, t, scalars);
  else
    hipLaunchKernelGGL(rmsprop_kernel, grid, dim3(256), 0, st, t, scalars);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_optim_step(int kind, int n_tensors, double* const* params,
                                const double* const* grads, double* const* exp_avg,
                                double* const* exp_avg_sq, const int64_t* sizes,
                                const double* scalars, void* stream) {
  return mepol_optim_step_snapshot(kind, n_tensors, params, grads, exp_avg, exp_avg_sq, sizes,
                                   scalars, nullptr, nullptr, nullptr, stream);
}
