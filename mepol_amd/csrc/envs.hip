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


// ---- whole rollout in one launch -----------------------------------------------------------
// One workgroup per trajectory runs all T steps of collect_particles (mepol.py:81-90) for the
// reference's 2-hidden-layer ReLU policy: x -> relu(W1 x + b1) -> relu(W2 h1 + b2) -> mean
// (policy.py:21-28, 53-61) -> a = mean + noise * exp(log_std) -> env step, with the states /
// actions recorded as f32.  Thread j owns hidden column j; its W1 row, biases and mean-layer
// column stay in registers, the first KL rows of W2^T (k-major, [h0][h1]) in LDS, and the rest
// of W2^T streams from L2 each step (coalesced: one 8-byte word per thread per k).  Replaces
// the per-step launch sequence (3 GEMMs + bias/ReLU + rollout_step, ~58 us per step even as a
// replayed graph) with ~3 barriers per step.
// Summation order: the layer-2 sum runs as kRollChunks fma chains over the row ranges
// [r L, r L + L), L = ceil(h0 / kRollChunks), combined as ((c0 + c1) + c2) + c3 -- exactly the
// multi-workgroup form's order (one chain per wave there), so both forms give the same bits
// and the host may pick either (or fall back from one to the other) per call.
constexpr int kRollMaxH = 512;
// mail word not yet published (memset 0xff): a NaN bit pattern no f64 partial sum of the
// policy's finite weights and activations produces
constexpr unsigned long long kMailEmpty = ~0ull;
constexpr int kRollMaxA = 8;
constexpr int kRollChunks = 4;

template <int ENV, int U>
__global__ __launch_bounds__(kRollMaxH) void rollout_mlp_kernel(
    const double* __restrict__ W1, const double* __restrict__ b1, int h0,
    const double* __restrict__ W2t, const double* __restrict__ b2, int h1,
    const double* __restrict__ Wm, const double* __restrict__ bm,
    const double* __restrict__ log_std, int a_dim, const double* __restrict__ init64,
    const float* __restrict__ init32, const double* __restrict__ noise, int64_t n, int64_t T,
    float* __restrict__ states_rec, float* __restrict__ actions_rec,
    double* __restrict__ visited, double* __restrict__ final_state, int KL) {
  extern __shared__ double sW2[];  // [KL][blockDim.x]: W2^T rows 0 .. KL - 1
  __shared__ double sx[2];
  __shared__ double sh1[kRollMaxH];
  __shared__ double spart[kRollMaxH / 64][kRollMaxA];
  const int64_t i = blockIdx.x;
  const int j = threadIdx.x, lane = j & 63, wave = j >> 6, nw = blockDim.x >> 6;
  const bool c0 = j < h0, c1 = j < h1;
  const double w1a = c0 ? W1[2 * j] : 0.0, w1b = c0 ? W1[2 * j + 1] : 0.0;
  const double bb1 = c0 ? b1[j] : 0.0, bb2 = c1 ? b2[j] : 0.0;
  double wm[kRollMaxA];
#pragma unroll
  for (int a = 0; a < kRollMaxA; ++a) wm[a] = (c1 && a < a_dim) ? Wm[a * h1 + j] : 0.0;
  for (int k = 0; k < KL; ++k) sW2[k * blockDim.x + j] = c1 ? W2t[(int64_t)k * h1 + j] : 0.0;
  const int L = (h0 + kRollChunks - 1) / kRollChunks;
  double p = 0.0, v = 0.0;  // MountainCar state (thread 0)
  float gx = 0.f, gy = 0.f;  // GridWorld state (thread 0)
  if (j == 0) {
    if (ENV == 0) {
      p = init64[2 * i];
      v = init64[2 * i + 1];
      sx[0] = p;
      sx[1] = v;
    } else {
      gx = init32[2 * i];
      gy = init32[2 * i + 1];
      sx[0] = (double)gx;
      sx[1] = (double)gy;
    }
    states_rec[(i * (T + 1)) * 2 + 0] = (float)sx[0];
    states_rec[(i * (T + 1)) * 2 + 1] = (float)sx[1];
  }
  // thread 0: exp(log_std) once, and the next step's noise loaded a step ahead (its global
  // latency would otherwise sit on the serial tail of every step)
  double sd[kRollMaxA], nz[kRollMaxA];
  if (j == 0) {
    for (int a = 0; a < a_dim; ++a) {
      sd[a] = exp(log_std[a]);
      nz[a] = noise[i * a_dim + a];
    }
  }
  __syncthreads();
  const double* col = W2t + (c1 ? j : 0);
  for (int64_t t = 0; t < T; ++t) {
    double nz_next[kRollMaxA];
    if (j == 0 && t + 1 < T)
      for (int a = 0; a < a_dim; ++a) nz_next[a] = noise[((t + 1) * n + i) * a_dim + a];
    // layer 1 (nf = 2)
    if (c0) sh1[j] = fmax(__dadd_rn(__dadd_rn(__dmul_rn(sx[0], w1a), __dmul_rn(sx[1], w1b)), bb1),
                          0.0);
    __syncthreads();
    // layer 2: h2_j = relu(sum_r c_r + b2[j]), c_r the fma chain over rows [r L, r L + L) in k
    // order; rows below KL come from LDS, the rest stream from L2 in batches of U loads with the
    // next batch in flight while this one is summed (L2 latency-bound: U rows per round trip)
    double acc = 0.0;
    for (int r = 0; r < kRollChunks; ++r) {
      const int ka = min(r * L, h0), kb = min(ka + L, h0);
      double c = 0.0;
      int k = ka;
      for (; k < min(kb, KL); ++k) c = fma(sW2[k * blockDim.x + j], sh1[k], c);
      double cur[U], nxt[U];
      const int kend = k + ((kb - k) / U) * U;
      if (k < kend) {
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = col[(int64_t)(k + u) * h1];
        for (; k < kend; k += U) {
          if (k + U < kend) {
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = col[(int64_t)(k + U + u) * h1];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) c = fma(c1 ? cur[u] : 0.0, sh1[k + u], c);
#pragma unroll
          for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
      }
      for (; k < kb; ++k) c = fma(c1 ? col[(int64_t)k * h1] : 0.0, sh1[k], c);
      acc = r == 0 ? c : acc + c;
    }
    const double h2 = c1 ? fmax(acc + bb2, 0.0) : 0.0;
    // mean layer: per-wave partial sums over its 64 columns, then waves in order
#pragma unroll
    for (int a = 0; a < kRollMaxA; ++a) {
      if (a < a_dim) {
        double q = wm[a] * h2;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m, kWave);
        if (lane == 0) spart[wave][a] = q;
      }
    }
    __syncthreads();
    if (j == 0) {
      double act[kRollMaxA];
      for (int a = 0; a < a_dim; ++a) {
        double mu = spart[0][a];
        for (int w = 1; w < nw; ++w) mu += spart[w][a];
        mu += bm[a];
        // output = mean + randn * exp(log_std)   (policy.py:59)
        act[a] = __dadd_rn(mu, __dmul_rn(nz[a], sd[a]));
        actions_rec[(i * T + t) * a_dim + a] = (float)act[a];
      }
      if (t + 1 < T)
        for (int a = 0; a < a_dim; ++a) nz[a] = nz_next[a];
      if (ENV == 0) {
        MountainCar::step(p, v, act[0]);
        sx[0] = p;
        sx[1] = v;
      } else {
        GridWorld::step(gx, gy, act[0], act[1]);
        sx[0] = (double)gx;
        sx[1] = (double)gy;
      }
      states_rec[(i * (T + 1) + t + 1) * 2 + 0] = (float)sx[0];
      states_rec[(i * (T + 1) + t + 1) * 2 + 1] = (float)sx[1];
      if (visited) {
        visited[(i * T + t) * 2 + 0] = sx[0];
        visited[(i * T + t) * 2 + 1] = sx[1];
      }
    }
    __syncthreads();
  }
  if (j == 0 && final_state) {
    final_state[2 * i] = sx[0];
    final_state[2 * i + 1] = sx[1];
  }
}

// ---- whole rollout, several workgroups per trajectory --------------------------------------
// rollout_mlp_kernel puts a trajectory on ONE CU, which then streams most of W2^T from L2 every
// step (11.7 us per step at C2's [300, 300]).  Here NP = ceil(h1 / 64) workgroups share a
// trajectory: workgroup p owns hidden-2 columns [64 p, 64 p + 64) and keeps their W2^T slice
// ([h0][64] f64, <= 154 KB) in LDS for all T steps.  Per step:
//   layer 1   all h0 columns (redundantly in every workgroup), 256 threads;
//   layer 2   its 64 columns; wave w of the 4 sums rows k in [w L, w L + L), L = ceil(h0 / 4), as
//             one fma chain (a single chain over 300 rows was 5.6 of the 8.4 us step:
//             tools/rollout_probe.py), and the column total is ((c0 + c1) + c2) + c3;
//   mean      wave 0's partial of the mean layer over its 64 columns (xor shuffle tree),
//             published as NP * a_dim self-validating 8-byte mail words (sc1 stores) and polled
//             with sc1 loads by wave 0 of every workgroup of the trajectory (bounded: err = 1);
//   env       every thread sums the NP partials in part order, adds bm and the noise and steps
//             the env (the same state in every thread).
// The order is oracle/native/rollout_kordered.c's with k_chunks = 4 (mepol_rollout_mlp_plan_info
// reports it).  Needs all n * NP workgroups resident at once (one per CU by LDS): the host
// launches it only when n * NP <= the CU count.
// PROBE (tools/variants/rollout_probe.hip only): thread 0 of each workgroup accumulates
// s_memtime spans of the step's phases into probe[blockIdx.x][8]; the product has PROBE = false.
constexpr int kRollMwWaves = kRollChunks;  // one layer-2 chain per wave
template <int ENV, bool PROBE = false>
__global__ __launch_bounds__(64 * kRollMwWaves) void rollout_mlp_mw_kernel(
    const double* __restrict__ W1, const double* __restrict__ b1, int h0,
    const double* __restrict__ W2t, const double* __restrict__ b2, int h1,
    const double* __restrict__ Wm, const double* __restrict__ bm,
    const double* __restrict__ log_std, int a_dim, const double* __restrict__ init64,
    const float* __restrict__ init32, const double* __restrict__ noise, int64_t n, int64_t T,
    float* __restrict__ states_rec, float* __restrict__ actions_rec,
    double* __restrict__ visited, double* __restrict__ final_state, int np, int nw,
    unsigned long long* __restrict__ mail, int* __restrict__ err, int* __restrict__ ticket,
    long long* __restrict__ probe) {
  extern __shared__ double sW2[];  // [h0][64]: W2^T rows, this part's 64 columns
  __shared__ double sh1[kRollMaxH];
  __shared__ double spart[kRollMwWaves][64];
  __shared__ double sword[64];
  __shared__ int sbad;
  long long pr[8] = {0, 0, 0, 0, 0, 0, 0, 0}, pt = 0;
  auto stamp = [&](int k, double dep) {
    if constexpr (PROBE) {
      // readfirstlane waits for dep's VALU result, so the stamp follows the phase's work
      const int sink = __builtin_amdgcn_readfirstlane(__double2hiint(dep));
      const long long now = (long long)__builtin_amdgcn_s_memtime();
      if (k >= 0) pr[k] += now - pt;
      pr[7] += sink & 1;
      pt = now;
    }
  };
  // (trajectory, part) from a dispatch-order ticket, not from blockIdx: when a workgroup takes
  // ticket t, every ticket below t is held by a running workgroup, so the parts a workgroup
  // waits for are either running or next in line for a free slot.  With the whole grid
  // resident (the host's occupancy check) all parts run at once; with fewer slots (another
  // kernel on the CUs) complete trajectories still finish and free theirs: no deadlock without
  // a cooperative launch.
  __shared__ int sticket;
  if (threadIdx.x == 0) sticket = atomicAdd(ticket, 1);
  __syncthreads();
  const int64_t i = sticket / np;
  const int p = sticket % np;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int j = 64 * p + lane;
  const bool c1 = j < h1;
  for (int k = wv; k < h0; k += kRollMwWaves)
    sW2[k * 64 + lane] = c1 ? W2t[(int64_t)k * h1 + j] : 0.0;
  // this wave's rows of the layer-2 sum (wave-uniform)
  const int L = (h0 + kRollMwWaves - 1) / kRollMwWaves;
  const int kb = min(wv * L, h0), len = min(kb + L, h0) - kb;
  constexpr int kU1 = kRollMaxH / (64 * kRollMwWaves);  // layer-1 columns per thread
  double w1a[kU1], w1b[kU1], bb1[kU1];
#pragma unroll
  for (int u = 0; u < kU1; ++u) {
    const int c = tid + 64 * kRollMwWaves * u;
    const bool ok = c < h0;
    w1a[u] = ok ? W1[2 * c] : 0.0;
    w1b[u] = ok ? W1[2 * c + 1] : 0.0;
    bb1[u] = ok ? b1[c] : 0.0;
  }
  const double bb2 = c1 ? b2[j] : 0.0;
  double wm[kRollMaxA], sd[kRollMaxA], nz[kRollMaxA], bmv[kRollMaxA];
#pragma unroll
  for (int a = 0; a < kRollMaxA; ++a) {
    wm[a] = (c1 && a < a_dim) ? Wm[a * h1 + j] : 0.0;
    bmv[a] = a < a_dim ? bm[a] : 0.0;
    sd[a] = a < a_dim ? exp(log_std[a]) : 0.0;
    nz[a] = a < a_dim ? noise[i * a_dim + a] : 0.0;
  }
  // env state, stepped identically by every thread of every part of the trajectory
  double pp = 0.0, vv = 0.0, x0, x1;
  float gx = 0.f, gy = 0.f;
  if (ENV == 0) {
    pp = init64[2 * i];
    vv = init64[2 * i + 1];
    x0 = pp;
    x1 = vv;
  } else {
    gx = init32[2 * i];
    gy = init32[2 * i + 1];
    x0 = (double)gx;
    x1 = (double)gy;
  }
  const bool rec = p == 0 && tid == 0;
  if (rec) {
    states_rec[(i * (T + 1)) * 2 + 0] = (float)x0;
    states_rec[(i * (T + 1)) * 2 + 1] = (float)x1;
  }
  if (tid == 0) sbad = 0;
  __syncthreads();
  if constexpr (PROBE) pr[6] = -(long long)__builtin_amdgcn_s_memrealtime();
  stamp(-1, 0.0);
  for (int64_t t = 0; t < T; ++t) {
    double nz_next[kRollMaxA];
    if (t + 1 < T)
      for (int a = 0; a < a_dim; ++a) nz_next[a] = noise[((t + 1) * n + i) * a_dim + a];
    // layer 1 (nf = 2), every column
#pragma unroll
    for (int u = 0; u < kU1; ++u) {
      const int c = tid + 64 * kRollMwWaves * u;
      if (c < h0)
        sh1[c] = fmax(__dadd_rn(__dadd_rn(__dmul_rn(x0, w1a[u]), __dmul_rn(x1, w1b[u])), bb1[u]),
                      0.0);
    }
    __syncthreads();
    stamp(0, sh1[lane]);
    // layer 2, this wave's rows of this part's columns: one fma chain in k order; the LDS
    // operands of the next 8 rows are loaded while these 8 are summed (constant offsets from
    // one base: no per-row address arithmetic)
    {
      constexpr int U = 8;
      const double* wp = sW2 + kb * 64 + lane;
      const double* hp = sh1 + kb;
      double acc = 0.0, wc[U], hc[U], wn[U], hn[U];
      int k = 0;
      if (len >= U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          wc[u] = wp[u * 64];
          hc[u] = hp[u];
        }
        for (; k + 2 * U <= len; k += U) {
#pragma unroll
          for (int u = 0; u < U; ++u) {
            wn[u] = wp[(k + U + u) * 64];
            hn[u] = hp[k + U + u];
          }
#pragma unroll
          for (int u = 0; u < U; ++u) acc = fma(wc[u], hc[u], acc);
#pragma unroll
          for (int u = 0; u < U; ++u) {
            wc[u] = wn[u];
            hc[u] = hn[u];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = fma(wc[u], hc[u], acc);
        k += U;
      }
      // the last < U rows: all loads issued, then the chain (one LDS round trip, not one per row)
#pragma unroll
      for (int u = 0; u < U - 1; ++u)
        if (k + u < len) {
          wc[u] = wp[(k + u) * 64];
          hc[u] = hp[k + u];
        }
#pragma unroll
      for (int u = 0; u < U - 1; ++u)
        if (k + u < len) acc = fma(wc[u], hc[u], acc);
      spart[wv][lane] = acc;
    }
    __syncthreads();
    unsigned long long* slot = mail + (i * T + t) * np * a_dim;
    if (wv == 0) {
      double s = spart[0][lane];
#pragma unroll
      for (int w = 1; w < kRollMwWaves; ++w) s += spart[w][lane];
      const double h2 = c1 ? fmax(s + bb2, 0.0) : 0.0;
      stamp(1, h2);
      // mean layer: this part's partial over its 64 columns (xor shuffle tree), lane 0's, to
      // this step's own mail words (pre-filled with kMailEmpty, which no partial can equal:
      // each word validates itself, no flag)
#pragma unroll
      for (int a = 0; a < kRollMaxA; ++a) {
        if (a < a_dim) {
          double q = wm[a] * h2;
#pragma unroll
          for (int m = 32; m >= 1; m >>= 1) q += __shfl_xor(q, m, kWave);
          if (lane == 0)
            __hip_atomic_store(slot + p * a_dim + a, __double_as_longlong(q), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      stamp(2, 0.0);
      // every part's partials of this step: lane l < np a_dim polls word l (part l / a_dim,
      // action l % a_dim) with sc1 loads until it is published
      const int nword = np * a_dim;
      unsigned spins = 0;
      unsigned long long v = 0;
      while (true) {
        if (lane < nword)
          v = __hip_atomic_load(slot + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!__ballot(lane < nword && v == kMailEmpty)) break;
        if (++spins > (1u << 24)) {
          if (lane == 0) {
            atomicExch(err, 1);
            sbad = 1;
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if constexpr (PROBE) pr[5] += spins;
      sword[lane] = __longlong_as_double(v);
      stamp(3, sword[lane]);
    }
    __syncthreads();
    if (sbad) return;  // workgroup-uniform: every wave leaves together
    double act[kRollMaxA];
    for (int a = 0; a < a_dim; ++a) {
      // the parts' words loaded together, then summed in part order
      constexpr int kMaxP = kRollMaxH / 64;
      double wq[kMaxP];
#pragma unroll
      for (int q = 0; q < kMaxP; ++q)
        if (q < np) wq[q] = sword[q * a_dim + a];
      double mu = wq[0];
#pragma unroll
      for (int q = 1; q < kMaxP; ++q)
        if (q < np) mu += wq[q];
      for (int q = np; q < nw; ++q) mu += 0.0;  // rollout_mlp_kernel's waves without columns
      mu += bmv[a];
      // output = mean + randn * exp(log_std)   (policy.py:59)
      act[a] = __dadd_rn(mu, __dmul_rn(nz[a], sd[a]));
      if (rec) actions_rec[(i * T + t) * a_dim + a] = (float)act[a];
    }
    if (t + 1 < T)
      for (int a = 0; a < a_dim; ++a) nz[a] = nz_next[a];
    if (ENV == 0) {
      MountainCar::step(pp, vv, act[0]);
      x0 = pp;
      x1 = vv;
    } else {
      GridWorld::step(gx, gy, act[0], act[1]);
      x0 = (double)gx;
      x1 = (double)gy;
    }
    if (rec) {
      states_rec[(i * (T + 1) + t + 1) * 2 + 0] = (float)x0;
      states_rec[(i * (T + 1) + t + 1) * 2 + 1] = (float)x1;
      if (visited) {
        visited[(i * T + t) * 2 + 0] = x0;
        visited[(i * T + t) * 2 + 1] = x1;
      }
    }
    stamp(4, x0);
  }
  if (rec && final_state) {
    final_state[2 * i] = x0;
    final_state[2 * i + 1] = x1;
  }
  if constexpr (PROBE) {
    pr[6] += (long long)__builtin_amdgcn_s_memrealtime();
    if (tid < 8) {
      long long v = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) v = tid == k ? pr[k] : v;
      probe[blockIdx.x * 8 + tid] = v;
    }
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

// env_id 0 = MountainCar (init64 [n,2] f64), 1 = GridWorld (init32 [n,2] f32).  The policy is
// nf = 2 -> [h0, h1] -> a_dim with ReLU: W1 [h0,2], b1, W2t = W2^T [h0,h1], b2, Wm [a,h1], bm,
// log_std [a]; noise [T,n,a_dim] f64.  Writes states_rec [n,T+1,2] f32, actions_rec [n,T,a] f32,
// visited [n,T,2] f64 (nullable), final_state [n,2] f64 (nullable).
// Workspace: word 0 = error flag (zeroed by every call that gets a workspace), then for the
// multi-workgroup form the mail [n][T][np][a_dim] 8-byte words (kMailEmpty).
static size_t rollout_mw_bytes(int64_t n, int64_t T, int h1, int a_dim) {
  const int64_t np = (h1 + 63) / 64;
  return 256 + (size_t)n * T * np * a_dim * 8;
}
// [h0][64] f64 slice (dynamic) + sh1, spart, sword (static, 6.5 KB) within 160 KB of LDS
static constexpr int kRollMwMaxH0 = 306;

template <int ENV>
static int rollout_mw_prepare() {
  static bool attr = false;
  if (!attr) {
    MEPOL_HIP(hipFuncSetAttribute((const void*)rollout_mlp_mw_kernel<ENV>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  kRollMwMaxH0 * 64 * (int)sizeof(double)));
    attr = true;
  }
  return 0;
}

// The multi-workgroup form's parts exchange partial sums every step.  Its workgroups take
// (trajectory, part) from a dispatch-order ticket (see the kernel), which makes the exchange
// deadlock-free whenever a trajectory's np parts fit on the device; it is chosen only when the
// occupancy of the kernel at this LDS size times the CU count holds the whole grid (all parts
// in flight at once).  Otherwise the one-workgroup form runs, which sums in the same order and
// so gives the same bits.  (Round 4 used hipLaunchCooperativeKernel for the co-residency; its
// dedicated queue crashed the process at exit under rocprofv3: HIP's teardown of that queue
// faulted inside libhsa-runtime64 after the profiler had shut its queue interception down,
// profiles/r5/rollout_exit_crash.txt.)
static int rollout_use_mw(int env_id, int64_t n, int h0, int h1, int a_dim) {
  const int np = (h1 + 63) / 64;
  const char* mw = getenv("MEPOL_ROLLOUT_MW");
  if (h0 > kRollMwMaxH0 || np * a_dim > 64 || (mw && mw[0] == '0')) return 0;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const size_t lds = (size_t)h0 * 64 * sizeof(double);
  int per_cu = 0;
  hipError_t e;
  if (env_id == 0) {
    if (rollout_mw_prepare<0>()) return 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rollout_mlp_mw_kernel<0>,
                                                     64 * kRollMwWaves, lds);
  } else {
    if (rollout_mw_prepare<1>()) return 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rollout_mlp_mw_kernel<1>,
                                                     64 * kRollMwWaves, lds);
  }
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n * np <= (int64_t)per_cu * cus;
}

extern "C" int mepol_rollout_mlp_plan_info(int64_t n, int h0, int h1, int a_dim,
                                           int* workgroups_per_traj, int* k_chunks) {
  if (n <= 0 || h0 <= 0 || h1 <= 0 || h0 > kRollMaxH || h1 > kRollMaxH || a_dim <= 0 ||
      a_dim > kRollMaxA || !workgroups_per_traj || !k_chunks) {
    set_error("mepol_rollout_mlp_plan_info: bad arguments");
    return kErrBadArg;
  }
  // (GridWorld and MountainCar kernels have the same resources: env 1 stands for both)
  const int mw = rollout_use_mw(1, n, h0, h1, a_dim);
  *workgroups_per_traj = mw ? (h1 + 63) / 64 : 1;
  *k_chunks = kRollChunks;  // both forms
  return 0;
}

extern "C" int mepol_rollout_mlp_workspace_size(int64_t n, int64_t T, int h0, int h1, int a_dim,
                                                size_t* bytes) {
  if (n < 0 || T < 0 || h0 <= 0 || h1 <= 0 || a_dim <= 0 || a_dim > kRollMaxA || !bytes) {
    set_error("mepol_rollout_mlp_workspace_size: bad arguments");
    return kErrBadArg;
  }
  // the mail only when the multi-workgroup form would run; the error word always
  *bytes = (n > 0 && rollout_use_mw(1, n, h0, h1, a_dim)) ? rollout_mw_bytes(n, T, h1, a_dim)
                                                          : 256;
  return 0;
}

template <int ENV>
static hipError_t rollout_mw_launch(const double* W1, const double* b1, int h0,
                                    const double* W2t, const double* b2, int h1, const double* Wm,
                                    const double* bm, const double* log_std, int a_dim,
                                    const double* init64, const float* init32,
                                    const double* noise, int64_t n, int64_t T, float* states_rec,
                                    float* actions_rec, double* visited, double* final_state,
                                    int np, int nw, unsigned long long* mail, int* err,
                                    int* ticket, hipStream_t st) {
  long long* probe = nullptr;
  hipLaunchKernelGGL((rollout_mlp_mw_kernel<ENV>), dim3((unsigned)(n * np)),
                     dim3(64 * kRollMwWaves), (unsigned)((size_t)h0 * 64 * sizeof(double)), st,
                     W1, b1, h0, W2t, b2, h1, Wm, bm, log_std, a_dim, init64, init32, noise, n, T,
                     states_rec, actions_rec, visited, final_state, np, nw, mail, err, ticket,
                     probe);
  return hipGetLastError();
}

extern "C" int mepol_rollout_mlp(int env_id, const double* W1, const double* b1, int h0,
                                 const double* W2t, const double* b2, int h1, const double* Wm,
                                 const double* bm, const double* log_std, int a_dim,
                                 const double* init64, const float* init32, const double* noise,
                                 int64_t n, int64_t T, float* states_rec, float* actions_rec,
                                 double* visited, double* final_state, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (n <= 0 || T <= 0) return 0;
  if (h0 <= 0 || h1 <= 0 || h0 > kRollMaxH || h1 > kRollMaxH || a_dim <= 0 ||
      a_dim > kRollMaxA || env_id < 0 || env_id > 1 || (env_id == 0 && !init64) ||
      (env_id == 1 && (!init32 || a_dim != 2)) || !W1 || !b1 || !W2t || !b2 || !Wm || !bm ||
      !log_std || !noise || !states_rec || !actions_rec ||
      (workspace && workspace_bytes < sizeof(int))) {
    set_error("mepol_rollout_mlp: bad arguments (hidden <= %d, a_dim <= %d)", kRollMaxH,
              kRollMaxA);
    return kErrBadArg;
  }
  const int threads = ((h0 > h1 ? h0 : h1) + 63) / 64 * 64;
  hipStream_t st = (hipStream_t)stream;
  int* err = (int*)workspace;
  if (err) MEPOL_HIP(hipMemsetAsync(err, 0, sizeof(int), st));  // whichever form runs
  {
    // several workgroups per trajectory when all of them can be resident at once
    const int np = (h1 + 63) / 64, nw = threads / 64;
    if (workspace && workspace_bytes >= rollout_mw_bytes(n, T, h1, a_dim) &&
        rollout_use_mw(env_id, n, h0, h1, a_dim)) {
      unsigned long long* mail = (unsigned long long*)((char*)workspace + 256);
      int* ticket = err + 1;  // word 1 of the 256-byte header: the dispatch-order counter
      MEPOL_HIP(hipMemsetAsync(ticket, 0, sizeof(int), st));
      // every mail word starts as kMailEmpty (all ones)
      MEPOL_HIP(hipMemsetAsync(mail, 0xff, (size_t)n * T * np * a_dim * 8, st));
      const hipError_t e =
          env_id == 0
              ? rollout_mw_launch<0>(W1, b1, h0, W2t, b2, h1, Wm, bm, log_std, a_dim, init64,
                                     init32, noise, n, T, states_rec, actions_rec, visited,
                                     final_state, np, nw, mail, err, ticket, st)
              : rollout_mw_launch<1>(W1, b1, h0, W2t, b2, h1, Wm, bm, log_std, a_dim, init64,
                                     init32, noise, n, T, states_rec, actions_rec, visited,
                                     final_state, np, nw, mail, err, ticket, st);
      if (e == hipSuccess) return 0;
      (void)hipGetLastError();  // launch refused: the one-workgroup form
    }
  }
  const dim3 g((unsigned)n);
  // W2^T rows kept in LDS, the rest streamed: up to ~150 KB (MEPOL_ROLLOUT_KL caps it)
  const char* klv = getenv("MEPOL_ROLLOUT_KL");
  int KL = (int)((150 * 1024) / ((size_t)threads * sizeof(double)));
  if (klv) KL = std::min(KL, atoi(klv));
  KL = std::max(0, std::min(KL, h0));
  const size_t lds = (size_t)KL * threads * sizeof(double);
#define MEPOL_ROLL(E, U)                                                                          \
  do {                                                                                            \
    static bool attr = false;                                                                     \
    if (!attr) {                                                                                  \
      MEPOL_HIP(hipFuncSetAttribute((const void*)rollout_mlp_kernel<E, U>,                        \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024));     \
      attr = true;                                                                                \
    }                                                                                             \
    hipLaunchKernelGGL((rollout_mlp_kernel<E, U>), g, dim3(threads), lds, st, W1, b1, h0, W2t, b2, \
                       h1, Wm, bm, log_std, a_dim, init64, init32, noise, n, T, states_rec,       \
                       actions_rec, visited, final_state, KL);                                    \
  } while (0)
  if (env_id == 0)
    MEPOL_ROLL(0, 8);
  else
    MEPOL_ROLL(1, 8);
#undef MEPOL_ROLL
  MEPOL_CHECK_LAUNCH();
  return 0;
}
