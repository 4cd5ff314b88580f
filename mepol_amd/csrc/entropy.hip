// Importance weights, Kozachenko-Leonenko entropy / KL estimate and their gradient on gfx950.
//
// Reference (src/algorithms/mepol.py):
//   compute_importance_weights  :114-139   u_{n,t} = exp(cumsum_t(logp_T - logp_B)), w = u / sum(u)
//   compute_entropy             :142-154   W_i = sum_{c<k} w[I[i,c]]      (I[:, :-1]: self + k-1)
//                                          V_i = D[i,k]^ns pi^(ns/2) / G
//                                          H   = -sum_i (W_i/k) log(W_i/(V_i+eps) + eps) + B
//   compute_kl                  :157-174   KL  = (1/N) sum_i log(k/(N W_i) + eps)
//   policy_update / backward    :268-281   autograd through gather -> normalise -> exp/cumsum.
//
// The backward is the closed form of that autograd chain:
//   g_i     = dH/dW_i = -(1/k) [ln(r_i + eps) + r_i/(r_i + eps)],  r_i = W_i/(V_i + eps)
//   gamma_j = sum_{(i,c<k): I[i,c] = j} g_i               (deterministic CSR transpose of I)
//   S       = sum_j gamma_j w_j
//   dH/dDelta_{n,s} = sum_{t>=s} (gamma_{n,t} - S) w_{n,t}  (segmented reverse scan)
// and is handed to torch autograd as the gradient of logp_T (the MLP backward stays in torch).
//
// Everything is f64 (the reference's dtype, src/utils/dtypes.py:3) and every reduction has a
// fixed order, so results are bitwise reproducible run to run.
//
// Particle layout: trajectory n owns particles [off[n], off[n+1]); logp/grad arrays are dense
// [nt, T_stride] with t < len_n = off[n+1]-off[n] (mepol.py:121-136, ragged via real lengths).
#include "common.hpp"

#include <algorithm>

namespace mepol {
namespace ent {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------------------
// IW forward: one wave per trajectory, chunked inclusive scan of Delta, then exp.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void iw_scan_kernel(const double* __restrict__ logp_t,
                                                      const double* __restrict__ logp_b,
                                                      int64_t nt, int64_t T_stride,
                                                      const int64_t* __restrict__ off,
                                                      double* __restrict__ u,
                                                      double* __restrict__ traj_sum) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + w;
  if (n >= nt) return;
  const int64_t p0 = off[n];
  const int64_t len = off[n + 1] - p0;
  const int64_t chunk = (len + 63) / 64;
  const int64_t b = l * chunk, e = min(len, b + chunk);
  const double* lt = logp_t + n * T_stride;
  const double* lb = logp_b + n * T_stride;
  // lane-local sum of its chunk
  double s = 0.0;
  for (int64_t t = b; t < e; ++t) s += lt[t] - lb[t];
  // exclusive wave scan of lane sums
  double incl = s;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const double o = __shfl_up(incl, m, kWave);
    if (l >= m) incl += o;
  }
  double run = incl - s;
  double usum = 0.0;
  for (int64_t t = b; t < e; ++t) {
    run += lt[t] - lb[t];
    const double x = exp(run);
    u[p0 + t] = x;
    usum += x;
  }
  usum = wave_sum(usum);
  if (l == 0) traj_sum[n] = usum;
}

// Deterministic block-redundant reduction of a short array (every block gets the same value).
__device__ double block_reduce_array(const double* __restrict__ a, int64_t n, double* sh) {
  // each thread adds a[tid], a[tid + bd], ... in that order; 8 loads in flight per step (the
  // sharded reverse scan sums every rank's gamma partials, ~12k values per block)
  double s = 0.0;
  const int64_t bd = blockDim.x;
  int64_t i = threadIdx.x;
  for (; i + 7 * bd < n; i += 8 * bd) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = a[i + u * bd];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  for (; i < n; i += bd) s += a[i];
  s = wave_sum(s);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = s;
  __syncthreads();
  double tot = 0.0;
  const int nw = blockDim.x >> 6;
  for (int i = 0; i < nw; ++i) tot += sh[i];
  __syncthreads();
  return tot;
}

__global__ __launch_bounds__(256) void iw_normalize_kernel(const double* __restrict__ u,
                                                           const double* __restrict__ traj_sum,
                                                           int64_t nt, int64_t N,
                                                           double* __restrict__ w,
                                                           double* __restrict__ Uout) {
  __shared__ double sh[4];
  const double U = block_reduce_array(traj_sum, nt, sh);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) w[i] = u[i] / U;
  if (i == 0 && Uout) *Uout = U;
}

// ---------------------------------------------------------------------------------------
// Entropy / KL forward: gather W, volumes, per-particle terms, block partial sums.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void entropy_fwd_kernel(
    const double* __restrict__ w, const int32_t* __restrict__ idxT, const double* __restrict__ D,
    int64_t N, int64_t N_w, int k, int kp1, double ns, double pi_ns2_over_G, double eps,
    double* __restrict__ W_out, double* __restrict__ g_out, double* __restrict__ partials) {
  __shared__ double sh[2][4];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  double th = 0.0, tk = 0.0;
  if (i < N) {
    // 8 neighbours at a time: their ids, then their weights, all in flight before the first
    // add (the per-neighbour loop serialised two dependent loads per neighbour); same order
    double Wi = 0.0;
    constexpr int kCh = 8;
    for (int c0 = 0; c0 < k; c0 += kCh) {
      int id[kCh];
#pragma unroll
      for (int u = 0; u < kCh; ++u) id[u] = idxT[(int64_t)min(c0 + u, k - 1) * N + i];
      double wv[kCh];
#pragma unroll
      for (int u = 0; u < kCh; ++u) wv[u] = w[id[u]];
#pragma unroll
      for (int u = 0; u < kCh; ++u)
        if (c0 + u < k) Wi += wv[u];
    }
    const double V = pow(D[i * kp1 + k], ns) * pi_ns2_over_G;
    const double r = Wi / (V + eps);
    const double lr = log(r + eps);
    th = (Wi / k) * lr;
    tk = log((double)k / ((double)N_w * Wi) + eps);
    W_out[i] = Wi;
    g_out[i] = -(1.0 / k) * (lr + r / (r + eps));
  }
  th = wave_sum(th);
  tk = wave_sum(tk);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
    sh[0][wv] = th;
    sh[1][wv] = tk;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x + 0] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    partials[2 * blockIdx.x + 1] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
  }
}

// out[0] = H = -sum(term) + B ; out[1] = KL (unclamped) = sum(kl_term)/N_w ;
// out[2] = sum(term) ; out[3] = sum(kl_term)  (raw sums for multi-rank reduction)
// vals (nullable, the graph iteration's control scalars): vals[0] = the H that out[0] held on
// entry (H(theta_t) of the previous pass), vals[1] = the new KL; out is then overwritten.
__global__ __launch_bounds__(256) void entropy_finalize_kernel(const double* __restrict__ partials,
                                                               int64_t nblocks, double B,
                                                               int64_t N_w,
                                                               double* __restrict__ out,
                                                               double* __restrict__ vals) {
  __shared__ double sh[4];
  double a = 0.0, b = 0.0;
  for (int64_t i = threadIdx.x; i < nblocks; i += blockDim.x) {
    a += partials[2 * i];
    b += partials[2 * i + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ double sb[4];
  if (l == 0) {
    sh[wv] = a;
    sb[wv] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double ta = sh[0] + sh[1] + sh[2] + sh[3];
    const double tb = sb[0] + sb[1] + sb[2] + sb[3];
    if (vals) {
      vals[0] = out[0];
      vals[1] = (1.0 / (double)N_w) * tb;
    }
    out[0] = -ta + B;
    out[1] = (1.0 / (double)N_w) * tb;
    out[2] = ta;
    out[3] = tb;
  }
}

// ---------------------------------------------------------------------------------------
// CSR transpose of I[:, :k] (built once per epoch: indices are fixed within an epoch).
// ---------------------------------------------------------------------------------------
// ---------------------------------------------------------------------------------------
// Backward.
// ---------------------------------------------------------------------------------------
// gamma_j = sum over CSR segment of g_i ; block partials of sum_j gamma_j w_j.
// 16 lanes per particle: the segment's ids are read coalesced and 16 gathers of g are in flight
// per lane group (one lane per particle with a serial loop over ~k ids was latency-bound at
// 85 us for C3).  Fixed order: lane sums over a stride of 16, then an xor tree.
constexpr int kGammaLanes = 16;
constexpr int64_t kGammaMaxBlocks = 2048;  // 8 blocks (32 waves) per CU: full occupancy
__global__ __launch_bounds__(256) void gamma_kernel(const double* __restrict__ g,
                                                    const double* __restrict__ w,
                                                    const int32_t* __restrict__ off,
                                                    const int32_t* __restrict__ rows, int64_t n,
                                                    double* __restrict__ gamma,
                                                    double* __restrict__ partials) {
  __shared__ double sh[4];
  const int sub = threadIdx.x & (kGammaLanes - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x / kGammaLanes;
  double s = 0.0;
  // grid-stride over particles (at most kGammaMaxBlocks partials for the reverse scan to read)
  for (int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kGammaLanes; j < n;
       j += stride) {
    double gj = 0.0;
    const int32_t b = off[j], e = off[j + 1];
    // 4 of the lane's ids, then their 4 gathers, in flight together (clamped reads of the
    // segment's last id past its end); the sum keeps the lane's order x = b + sub, +16, ...
    for (int32_t x0 = b + sub; x0 < e; x0 += 4 * kGammaLanes) {
      int32_t r[4];
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) r[u] = rows[min(x0 + u * kGammaLanes, e - 1)];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = g[r[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (x0 + u * kGammaLanes < e) gj += v[u];
    }
#pragma unroll
    for (int m = kGammaLanes / 2; m >= 1; m >>= 1) gj += __shfl_xor(gj, m, kWave);
    if (sub == 0) {
      gamma[j] = gj;
      s += gj * w[j];
    }
  }
  s = wave_sum(s);
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[wv] = s;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// grad_logp[n, s] = gH * sum_{t >= s} (gamma_{n,t} - S) w_{n,t} ; S = sum(partials) (or *S_ext).
__global__ __launch_bounds__(256) void reverse_scan_kernel(
    const double* __restrict__ gamma, const double* __restrict__ w,
    const double* __restrict__ partials, int64_t nparts, const double* __restrict__ S_ext,
    const int64_t* __restrict__ off, int64_t nt, int64_t T_stride,
    const double* __restrict__ gH, double* __restrict__ grad_logp) {
  __shared__ double sh[4];
  const double S = S_ext ? *S_ext : block_reduce_array(partials, nparts, sh);
  const double up = *gH;
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int64_t n = (int64_t)blockIdx.x * 4 + wv;
  if (n >= nt) return;
  const int64_t p0 = off[n];
  const int64_t len = off[n + 1] - p0;
  const int64_t chunk = (len + 63) / 64;
  const int64_t b = l * chunk, e = min(len, b + chunk);
  double s = 0.0;
  for (int64_t t = e - 1; t >= b; --t) s += (gamma[p0 + t] - S) * w[p0 + t];
  // exclusive suffix scan over lanes (lanes above contribute)
  double incl = s;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const double o = __shfl_down(incl, m, kWave);
    if (l + m < 64) incl += o;
  }
  double run = incl - s;
  double* gout = grad_logp + n * T_stride;
  for (int64_t t = e - 1; t >= b; --t) {
    run += (gamma[p0 + t] - S) * w[p0 + t];
    gout[t] = up * run;
  }
  // zero the padded tail of a ragged trajectory
  for (int64_t t = len + l; t < T_stride; t += 64) gout[t] = 0.0;
}

}  // namespace ent
}  // namespace mepol

using namespace mepol;
using namespace mepol::ent;

extern "C" int mepol_iw_forward(const double* logp_t, const double* logp_b, int64_t num_traj,
                                int64_t T_stride, const int64_t* traj_offsets, int64_t n_particles,
                                double* u_out, double* traj_sum_out, double* w_out, double* U_out,
                                void* stream) {
  if (num_traj <= 0 || T_stride <= 0 || !logp_t || !logp_b || !traj_offsets || !u_out ||
      !traj_sum_out) {
    set_error("mepol_iw_forward: bad arguments");
    return kErrBadArg;
  }
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(iw_scan_kernel, dim3((unsigned)((num_traj + 3) / 4)), dim3(256), 0, st, logp_t,
                     logp_b, num_traj, T_stride, traj_offsets, u_out, traj_sum_out);
  MEPOL_CHECK_LAUNCH();
  if (w_out) {
    hipLaunchKernelGGL(iw_normalize_kernel, dim3((unsigned)((n_particles + 255) / 256)), dim3(256), 0,
                       st, u_out, traj_sum_out, num_traj, n_particles, w_out, U_out);
    MEPOL_CHECK_LAUNCH();
  }
  return 0;
}

// Normalise u by an externally supplied total (multi-rank: U = all-reduce of local sums).
__global__ void scale_by_kernel(const double* __restrict__ u, const double* __restrict__ U,
                                int64_t n, double* __restrict__ w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) w[i] = u[i] / *U;
}

extern "C" int mepol_iw_normalize(const double* u, const double* U, int64_t n, double* w,
                                  void* stream) {
  hipLaunchKernelGGL(scale_by_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, u, U, n, w);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_entropy_partials_size(int64_t n_particles) {
  return (int)((n_particles + kBlock - 1) / kBlock);
}

// w: [N_w] (all particles, global indexing); idxT: [kp1][n] transposed neighbour indices of the
// n local query particles; D: [n][kp1].  out4 = {H, KL_unclamped, sum term, sum kl_term}.
static int entropy_forward_impl(const double* w, const int32_t* idxT, const double* D, int64_t n,
                                int64_t n_w, int k, int kp1, double ns, double G, double B,
                                double eps, double* W_out, double* g_out, double* partials,
                                double* out4, double* vals, void* stream) {
  if (n < 0 || k <= 0 || kp1 <= k || !w || !idxT || !D || !W_out || !g_out || !partials || !out4) {
    set_error("mepol_entropy_forward: bad arguments");
    return kErrBadArg;
  }
  hipStream_t st = (hipStream_t)stream;
  const int64_t nb = (n + kBlock - 1) / kBlock;
  const double pi_ns2_over_G = pow(M_PI, ns / 2.0) / G;
  if (nb > 0) {
    hipLaunchKernelGGL(entropy_fwd_kernel, dim3((unsigned)nb), dim3(kBlock), 0, st, w, idxT, D, n,
                       n_w, k, kp1, ns, pi_ns2_over_G, eps, W_out, g_out, partials);
    MEPOL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(entropy_finalize_kernel, dim3(1), dim3(256), 0, st, partials, nb, B, n_w, out4,
                     vals);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_entropy_forward(const double* w, const int32_t* idxT, const double* D,
                                     int64_t n, int64_t n_w, int k, int kp1, double ns, double G,
                                     double B, double eps, double* W_out, double* g_out,
                                     double* partials, double* out4, void* stream) {
  return entropy_forward_impl(w, idxT, D, n, n_w, k, kp1, ns, G, B, eps, W_out, g_out, partials,
                              out4, nullptr, stream);
}

// The graph iteration's form: out4 is updated in place and vals = {H held on entry, new KL}
// (the two control scalars the host reads), with no separate stack / copy launches.
extern "C" int mepol_entropy_forward_emit(const double* w, const int32_t* idxT, const double* D,
                                          int64_t n, int64_t n_w, int k, int kp1, double ns,
                                          double G, double B, double eps, double* W_out,
                                          double* g_out, double* partials, double* out4,
                                          double* vals, void* stream) {
  if (!vals) {
    set_error("mepol_entropy_forward_emit: vals is null");
    return kErrBadArg;
  }
  return entropy_forward_impl(w, idxT, D, n, n_w, k, kp1, ns, G, B, eps, W_out, g_out, partials,
                              out4, vals, stream);
}

// The block partials mepol_entropy_gamma writes for n_own particles (its reverse scan reads them).
extern "C" int mepol_entropy_gamma_partials_size(int64_t n_own) {
  return (int)std::min<int64_t>((n_own * kGammaLanes + 255) / 256, kGammaMaxBlocks);
}

// gamma over the n_own particles this rank owns (CSR over its own ids), partial S per block.
extern "C" int mepol_entropy_gamma(const double* g, const double* w_own, const int32_t* csr_off,
                                   const int32_t* csr_rows, int64_t n_own, double* gamma_out,
                                   double* partials, void* stream) {
  const int64_t nb = std::min<int64_t>((n_own * kGammaLanes + 255) / 256, kGammaMaxBlocks);
  if (nb == 0) return 0;
  hipLaunchKernelGGL(gamma_kernel, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, g, w_own,
                     csr_off, csr_rows, n_own, gamma_out, partials);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

// grad_logp [nt, T_stride] from gamma / w of the local trajectories.  S is either reduced from
// `partials` (nparts of them, single-rank) or read from S_ext (multi-rank all-reduced value).
extern "C" int mepol_entropy_reverse_scan(const double* gamma, const double* w,
                                          const double* partials, int64_t nparts,
                                          const double* S_ext, const int64_t* traj_offsets,
                                          int64_t num_traj, int64_t T_stride, const double* grad_H,
                                          double* grad_logp, void* stream) {
  if (num_traj <= 0) return 0;
  hipLaunchKernelGGL(reverse_scan_kernel, dim3((unsigned)((num_traj + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, gamma, w, partials, nparts, S_ext, traj_offsets, num_traj,
                     T_stride, grad_H, grad_logp);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

// ---- sharded iteration helpers (parallel.py ShardedIteration, one launch each) -------------
// w_glob[r n + i] = xu_all[r (n + nt) + i] / U, U = the sum of the world * nt trajectory sums
// xu_all[r (n + nt) + n + t]: the all-gathered [u | trajectory sums] blocks of every rank
// normalised in one pass.  Every block forms U with the same fixed tree (a strided partial per
// thread, then pairwise in LDS), so every block of every rank holds the same bits.
constexpr int kGatherThreads = 256;
__global__ __launch_bounds__(kGatherThreads) void iw_normalize_gathered_kernel(
    const double* __restrict__ xu_all, int world, int64_t n, int nt, double* __restrict__ w_glob) {
  __shared__ double red[kGatherThreads];
  const int tid = threadIdx.x;
  const int64_t tot = (int64_t)world * nt;
  double p = 0.0;
  for (int64_t e = tid; e < tot; e += kGatherThreads) {
    const int64_t r = e / nt, t = e % nt;
    p += xu_all[r * (n + nt) + n + t];
  }
  red[tid] = p;
  __syncthreads();
  for (int s = kGatherThreads / 2; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const double U = red[0];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + tid;
  if (e >= (int64_t)world * n) return;
  const int64_t r = e / n, i = e % n;
  w_glob[e] = xu_all[r * (n + nt) + i] / U;
}

// The two control scalars of a sharded replay from the all-gathered raw sums (stride apart,
// at offset off of each rank's block): sums = rank-order sums, vals = {B - sums_cur[0] (the H
// of the previous pass), sums[1] / N_global (the new KL)}, then sums_cur = sums.
__global__ void sharded_emit_kernel(const double* __restrict__ x_all, int world, int64_t stride,
                                    int64_t off, double B, int64_t n_global,
                                    double* __restrict__ sums_cur, double* __restrict__ vals) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double s0 = 0.0, s1 = 0.0;
  for (int r = 0; r < world; ++r) {
    s0 += x_all[(int64_t)r * stride + off];
    s1 += x_all[(int64_t)r * stride + off + 1];
  }
  vals[0] = B - sums_cur[0];
  vals[1] = s1 / (double)n_global;
  sums_cur[0] = s0;
  sums_cur[1] = s1;
}

extern "C" int mepol_iw_normalize_gathered(const double* xu_all, int world, int64_t n, int nt,
                                           double* w_glob, void* stream) {
  if (world <= 0 || n <= 0 || nt <= 0 || !xu_all || !w_glob) {
    set_error("mepol_iw_normalize_gathered: bad arguments");
    return kErrBadArg;
  }
  const int64_t tot = (int64_t)world * n;
  hipLaunchKernelGGL(iw_normalize_gathered_kernel,
                     dim3((unsigned)((tot + kGatherThreads - 1) / kGatherThreads)),
                     dim3(kGatherThreads), 0, (hipStream_t)stream, xu_all, world, n, nt, w_glob);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_sharded_emit(const double* x_all, int world, int64_t stride, int64_t off,
                                  double B, int64_t n_global, double* sums_cur, double* vals,
                                  void* stream) {
  if (world <= 0 || off + 1 >= stride || !x_all || !sums_cur || !vals) {
    set_error("mepol_sharded_emit: bad arguments");
    return kErrBadArg;
  }
  hipLaunchKernelGGL(sharded_emit_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, x_all, world,
                     stride, off, B, n_global, sums_cur, vals);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
