// Batched environment steppers for the MEPOL rollout (collect_particles, mepol.py:70-111).
//
//  MountainCar   src/envs/mountain_car_wall.py:13-45 (+ gym 0.17.2 Continuous_MountainCarEnv
//                constants: position in [-1.2, 0.6], |v| <= 0.07, power 0.0015, goal 0.45).
//                State is f64 (np.array([position, velocity]), :44).
//  GridWorld     src/envs/gridworld_continuous.py:128-154, walls :66-76.  State is f32
//                (:150); the move is evaluated in f64 (f32 state + f64 clipped action).
//  ErgodicEnv    src/envs/wrappers.py:12-15: done is always False, every trajectory runs T steps.
//
// Each step is evaluated with the same IEEE operations, in the same order, as the reference's
// numpy/Python scalar code (explicit _rn intrinsics: no contraction), so a step is bit-exact
// except for cos() in MountainCar, whose last-ulp rounding may differ from glibc.
//
// The fused rollout step takes the policy mean from the PyTorch MLP and Gaussian noise, forms
// a = mean + noise * exp(log_std) (policy.py:59), records (s_t, a_t) as f32 (mepol.py:74-75,
// 82-86) and advances the env state, all in one launch per step.
#include "common.hpp"

namespace mepol {
namespace envs {

struct MountainCar {
  static constexpr double kMinPos = -1.2, kMaxPos = 0.6, kMaxSpeed = 0.07, kGoal = 0.45;
  static constexpr double kPower = 0.0015;
  __device__ static void step(double& p, double& v, double a0) {
    const double force = fmin(fmax(a0, -1.0), 1.0);
    // velocity += force*power - 0.0025*cos(3*position)
    const double t1 = __dmul_rn(force, kPower);
    const double t2 = __dmul_rn(0.0025, cos(__dmul_rn(3.0, p)));
    v = __dadd_rn(v, __dsub_rn(t1, t2));
    if (v > kMaxSpeed) v = kMaxSpeed;
    if (v < -kMaxSpeed) v = -kMaxSpeed;
    p = __dadd_rn(p, v);
    if (p > kMaxPos) p = kMaxPos;
    if (p < kMinPos) p = kMinPos;
    if (p == kMinPos && v < 0) v = 0.0;
    if (p > kGoal) {
      p = kGoal;
      v = 0.0;
    }
  }
};

struct GridWorld {
  static constexpr double kDim = 6.0, kMaxDelta = 0.2, kWall = 2.5;
  __device__ static bool inside(double x, double y, double x0, double x1, double y0, double y1) {
    return x0 <= x && x <= x1 && y0 <= y && y <= y1;
  }
  __device__ static void step(float& sx, float& sy, double ax, double ay) {
    const double dx = fmin(fmax(ax, -kMaxDelta), kMaxDelta);
    const double dy = fmin(fmax(ay, -kMaxDelta), kMaxDelta);
    const double x = (double)sx, y = (double)sy;
    double nx = __dadd_rn(x, dx), ny = __dadd_rn(y, dy);
    constexpr double h = kWall / 2;
    bool hit = inside(nx, ny, -h, h, -kWall, kWall) || inside(nx, ny, -kWall, -h, -h, h) ||
               inside(nx, ny, h, kWall, -h, h) || inside(nx, ny, -kDim, -(kDim - kWall), -h, h) ||
               inside(nx, ny, -h, h, -kDim, -(kDim - kWall)) ||
               inside(nx, ny, kDim - kWall, kDim, -h, h) ||
               inside(nx, ny, -h, h, kDim - kWall, kDim);
    if (hit) {
      nx = x;
      ny = y;
    }
    if (fabs(nx) >= kDim || fabs(ny) >= kDim) {
      nx = x;
      ny = y;
    }
    sx = (float)nx;
    sy = (float)ny;
  }
};

__global__ void step_mc_kernel(double* __restrict__ s, const double* __restrict__ a, int64_t n,
                               int64_t a_stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double p = s[2 * i], v = s[2 * i + 1];
  MountainCar::step(p, v, a[i * a_stride]);
  s[2 * i] = p;
  s[2 * i + 1] = v;
}

__global__ void step_gw_kernel(float* __restrict__ s, const double* __restrict__ a, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = s[2 * i], y = s[2 * i + 1];
  GridWorld::step(x, y, a[2 * i], a[2 * i + 1]);
  s[2 * i] = x;
  s[2 * i + 1] = y;
}

// One rollout step for n trajectories.  env_f64: MountainCar state [n,2] (f64);
// env_f32: GridWorld state [n,2] (f32).  policy_in [n,2] f64 receives the next policy input.
// states_rec [n, T+1, 2] f32, actions_rec [n, T, a_dim] f32.
template <int ENV>
__global__ void rollout_step_kernel(double* __restrict__ env_f64, float* __restrict__ env_f32,
                                    const double* __restrict__ mean,
                                    const double* __restrict__ noise,
                                    const double* __restrict__ log_std, int64_t n, int a_dim,
                                    int64_t t, int64_t T, float* __restrict__ states_rec,
                                    float* __restrict__ actions_rec,
                                    double* __restrict__ policy_in) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double act[8];
  for (int j = 0; j < a_dim && j < 8; ++j) {
    // output = mean + randn * exp(log_std)   (policy.py:59)
    act[j] = __dadd_rn(mean[i * a_dim + j], __dmul_rn(noise[i * a_dim + j], exp(log_std[j])));
    actions_rec[(i * T + t) * a_dim + j] = (float)act[j];
  }
  if (ENV == 0) {
    double p = env_f64[2 * i], v = env_f64[2 * i + 1];
    MountainCar::step(p, v, act[0]);
    env_f64[2 * i] = p;
    env_f64[2 * i + 1] = v;
    policy_in[2 * i] = p;
    policy_in[2 * i + 1] = v;
    states_rec[(i * (T + 1) + t + 1) * 2 + 0] = (float)p;
    states_rec[(i * (T + 1) + t + 1) * 2 + 1] = (float)v;
  } else {
    float x = env_f32[2 * i], y = env_f32[2 * i + 1];
    GridWorld::step(x, y, act[0], act[1]);
    env_f32[2 * i] = x;
    env_f32[2 * i + 1] = y;
    policy_in[2 * i] = (double)x;
    policy_in[2 * i + 1] = (double)y;
    states_rec[(i * (T + 1) + t + 1) * 2 + 0] = x;
    states_rec[(i * (T + 1) + t + 1) * 2 + 1] = y;
  }
}

}  // namespace envs
}  // namespace mepol

using namespace mepol;
using namespace mepol::envs;

extern "C" int mepol_step_mountaincar(double* state, const double* action, int64_t n,
                                      int64_t action_stride, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(step_mc_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, state, action, n, action_stride);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_step_gridworld(float* state, const double* action, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(step_gw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, state, action, n);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

// env_id: 0 = MountainCar (env_f64 state), 1 = GridWorld (env_f32 state).
extern "C" int mepol_rollout_step(int env_id, double* env_f64, float* env_f32, const double* mean,
                                  const double* noise, const double* log_std, int64_t n, int a_dim,
                                  int64_t t, int64_t T, float* states_rec, float* actions_rec,
                                  double* policy_in, void* stream) {
  if (n <= 0) return 0;
  if (a_dim <= 0 || a_dim > 8 || t < 0 || t >= T || (env_id == 0 && !env_f64) ||
      (env_id == 1 && (!env_f32 || a_dim != 2)) || env_id < 0 || env_id > 1) {
    set_error("mepol_rollout_step: bad arguments (env %d, a_dim %d, t %lld)", env_id, a_dim,
              (long long)t);
    return kErrBadArg;
  }
  hipStream_t st = (hipStream_t)stream;
  dim3 g((unsigned)((n + 255) / 256));
  if (env_id == 0)
    hipLaunchKernelGGL(rollout_step_kernel<0>, g, dim3(256), 0, st, env_f64, env_f32, mean, noise,
                       log_std, n, a_dim, t, T, states_rec, actions_rec, policy_in);
  else
    hipLaunchKernelGGL(rollout_step_kernel<1>, g, dim3(256), 0, st, env_f64, env_f32, mean, noise,
                       log_std, n, a_dim, t, T, states_rec, actions_rec, policy_in);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
