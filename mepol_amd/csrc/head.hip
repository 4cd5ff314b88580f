// Fused Gaussian policy head: mean layer + log-probability (GaussianPolicy.get_log_p,
// src/policy.py:43-51) and its backward, with the last hidden layer's ReLU folded in.
//
// forward : h = relu(z);  mu = h Wm^T + bm;  sigma = exp(log_std) + 1e-7
//           logp_i = sum_a -0.5 (log 2pi + 2 log_std_a + (act_ia - mu_ia)^2 / sigma_a^2)
// backward: dmu_ia = g_i (act_ia - mu_ia) / sigma_a^2
//           dlog_std_a = sum_i g_i (-1 + (act_ia - mu_ia)^2 exp(log_std_a) / sigma_a^3)
//           dbm_a = sum_i dmu_ia ;  dWm_ac = sum_i dmu_ia h_ic
//           dz_ic = (sum_a dmu_ia Wm_ac) [z_ic > 0]        (ReLU backward fused)
// One wave per row: z rows are read once, coalesced (64 lanes x 8 B); Wm stays in LDS.  This
// replaces the PyTorch sequence mean-GEMM, 6 elementwise kernels and a reduction in the forward,
// and dX-GEMM, dW-GEMM, threshold_backward and the elementwise chain in the backward: the head
// is HBM-bound (one pass over z forward; z read + dz written backward).
// Reductions over rows go through per-block partials summed in a fixed order (deterministic).
#include "common.hpp"

#include <algorithm>

namespace mepol {
namespace head {

#ifndef MEPOL_HEAD_BWD_PF
#define MEPOL_HEAD_BWD_PF 1  // rows prefetched per wave in head_bwd_kernel
#endif

constexpr int kMaxA = 32;     // fused path: action_dim <= 32 (MC 1, GW 2, Ant 8, Humanoid 17, HandReach 20)
constexpr int kMaxCols = 8;   // columns per lane: hidden <= 512
constexpr double kLog2Pi = 1.8378770664093453;
constexpr double kStdEps = 1e-7;

// Reduce-scatter of AP per-lane values over groups of G lanes (G a power of two <= 64, lanes
// of a group consecutive): halving exchanges, then a butterfly over the remaining lanes.  Lane
// l ends with the group's sum for component a_out; lanes of a group agreeing on the bits
// log2(G)-1 .. log2(G)-log2(AP) hold the same component.
template <int AP, int G>
__device__ __forceinline__ double reduce_scatter_g(double (&v)[AP], int l, int& a_out) {
  double cur[AP];
#pragma unroll
  for (int a = 0; a < AP; ++a) cur[a] = v[a];
  int a_idx = 0;
  int len = AP;
  int bit = G / 2;
#pragma unroll
  for (int step = AP; step > 1; step >>= 1) {
    const bool upper = (l & bit) != 0;
    const int half = len >> 1;
#pragma unroll
    for (int a = 0; a < AP / 2; ++a) {
      if (a < half) {
        const double send = upper ? cur[a] : cur[a + half];
        const double keep = upper ? cur[a + half] : cur[a];
        cur[a] = keep + __shfl_xor(send, bit, kWave);
      }
    }
    a_idx = a_idx * 2 + (upper ? 1 : 0);
    len = half;
    bit >>= 1;
  }
  double x = cur[0];
  for (; bit >= 1; bit >>= 1) x += __shfl_xor(x, bit, kWave);
  a_out = a_idx;
  return x;
}

// Forward with 16 lanes per row and 4 rows per wave: lane (r = l>>4, q = l&15) owns columns
// c = q + 16 j (j < NCL) of row 4 i + r.  Each lane runs NCL x AP fma into AP accumulators; the
// cross-lane reduction is over 16 lanes (4 exchange steps for all AP components) and is shared
// by 4 rows, so the per-row VALU work is ~H*AP/16 fma + a few exchanges (the 64-lanes-per-row
// form spent most of its time in the 64-lane reduction and its selects).  Wm, bz and the
// per-component constants live in LDS; loads of z are 4 rows x 128 B segments, next group
// prefetched.
template <int AP, int NCL, int NCH>
__global__ __launch_bounds__(256) void head_fwd16_kernel(
    const double* __restrict__ z, int64_t N, int H, const double* __restrict__ bz,
    const double* __restrict__ Wm, const double* __restrict__ bm,
    const double* __restrict__ log_std, const double* __restrict__ act, int A,
    double* __restrict__ mu_out, double* __restrict__ logp_out) {
  constexpr int AP2 = AP >= 2 ? AP / 2 : 1;
  constexpr int APT = AP * NCH;                // action slots (chunks of AP)
  __shared__ double2 sW2[NCH * NCL * AP2 * 16];  // [chunk][j][a/2][q] pairs (a even, a+1)
  __shared__ double sB[NCL * 16];                // [j][q] folded bias of z
  __shared__ double sK[3][APT];                  // bm, log 2pi + 2 log_std, 1/sigma^2
  const int l = threadIdx.x & 63;
  const int q = l & 15, r = l >> 4;
  for (int e = threadIdx.x; e < NCH * NCL * AP2 * 16; e += blockDim.x) {
    const int qq = e & 15, a2 = (e >> 4) % AP2, j = ((e >> 4) / AP2) % NCL;
    const int ch = (e >> 4) / (AP2 * NCL);
    const int c = qq + 16 * j;
    const int a0 = ch * AP + 2 * a2, a1 = a0 + 1;
    double2 w;
    w.x = (c < H && a0 < A) ? Wm[a0 * H + c] : 0.0;
    w.y = (AP >= 2 && c < H && a1 < A) ? Wm[a1 * H + c] : 0.0;
    sW2[e] = w;
  }
  for (int e = threadIdx.x; e < NCL * 16; e += blockDim.x) sB[e] = (bz && e < H) ? bz[e] : 0.0;
  if (threadIdx.x < APT) {
    const int a = threadIdx.x;
    const double lsa = (a < A) ? log_std[a] : 0.0;
    const double sd = exp(lsa) + kStdEps;
    sK[0][a] = (a < A) ? bm[a] : 0.0;
    sK[1][a] = kLog2Pi + 2.0 * lsa;
    sK[2][a] = 1.0 / (sd * sd);
  }
  __syncthreads();
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t ngroups = (N + 3) / 4;
  double zn[NCL];
  const int64_t last = N - 1;
  auto load_group = [&](int64_t gi) {  // clamped, unconditional loads (see head_bwd_kernel)
    const int64_t row = gi * 4 + r;
    const double* zr = z + (row < N ? row : last) * H;
#pragma unroll
    for (int j = 0; j < NCL; ++j) {
      const int c = q + 16 * j;
      zn[j] = zr[c < H ? c : H - 1];
    }
  };
  const int64_t wave_u = __builtin_amdgcn_readfirstlane((int)wave);
  load_group(wave_u);
  for (int64_t gi = wave_u; gi < ngroups; gi += nwaves) {
    double zc[NCL];
#pragma unroll
    for (int j = 0; j < NCL; ++j) zc[j] = zn[j];
    load_group(gi + nwaves);
    const int64_t row = gi * 4 + r;
    int qo = q;
    asm volatile("" : "+v"(qo));  // keep the LDS reads inside the loop
    if (NCH > 1) {  // relu(z + b) once, reused by every chunk
#pragma unroll
      for (int j = 0; j < NCL; ++j) zc[j] = fmax(zc[j] + sB[j * 16 + qo], 0.0);
    }
    // lanes of a row with equal component: (16 / AP) of them; the lowest one writes
    const bool writer = (q & ((16 / AP) - 1)) == 0;
    double term = 0.0;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      double acc[AP];
#pragma unroll
      for (int a = 0; a < AP; ++a) acc[a] = 0.0;
#pragma unroll
      for (int j = 0; j < NCL; ++j) {
        const double x = NCH > 1 ? zc[j] : fmax(zc[j] + sB[j * 16 + qo], 0.0);
#pragma unroll
        for (int a2 = 0; a2 < AP2; ++a2) {
          const double2 w = sW2[((ch * NCL + j) * AP2 + a2) * 16 + qo];
          acc[2 * a2] = fma(x, w.x, acc[2 * a2]);
          if (AP >= 2) acc[2 * a2 + 1] = fma(x, w.y, acc[2 * a2 + 1]);
        }
      }
      int ac;
      const double v = reduce_scatter_g<AP, 16>(acc, l, ac);
      const int a = ch * AP + ac;
      if (row < N && a < A && writer) {
        const double m = v + sK[0][a];
        const double d = act[row * A + a] - m;
        mu_out[row * A + a] = m;
        term += -0.5 * (sK[1][a] + d * d * sK[2][a]);
      }
    }
    // logp_row = sum over the row's 16 lanes (non-writers hold 0)
#pragma unroll
    for (int bit = 8; bit >= 1; bit >>= 1) term += __shfl_xor(term, bit, kWave);
    if (q == 0 && row < N) logp_out[row] = term;
  }
}

// v from lane `lane` into an SGPR pair (wave-uniform).
__device__ __forceinline__ double readlane_d(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Per-block partial records [dW (A*H) | db (A) | dls (A)], reduced by reduce_partials_kernel.
template <int AP, int NC>
__global__ __launch_bounds__(256) void head_bwd_kernel(
    const double* __restrict__ gl, const double* __restrict__ z, int64_t N, int H,
    const double* __restrict__ bz, const double* __restrict__ Wm, const double* __restrict__ log_std,
    const double* __restrict__ act, const double* __restrict__ mu, int A,
    double* __restrict__ dz, double* __restrict__ part) {
  __shared__ double sW[NC * 64 * AP];   // [j][a][lane]
  __shared__ double sRed[AP * 64 * NC + 64 * NC];  // block accumulators, waves add in order 0..3
  __shared__ double sb[4][AP], sls[4][AP];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int e = threadIdx.x; e < NC * 64 * AP; e += blockDim.x) {
    const int ll = e & 63, a = (e >> 6) % AP, j = (e >> 6) / AP;
    const int c = ll + 64 * j;
    sW[e] = (c < H && a < A) ? Wm[a * H + c] : 0.0;
  }
  __syncthreads();
  double es3 = 0.0, inv = 0.0;  // lane a (< A) owns component a of dmu / db / dlog_std
  if (l < A) {
    const double e = exp(log_std[l]);
    const double sd = e + kStdEps;
    es3 = e / (sd * sd * sd);
    inv = 1.0 / (sd * sd);
  }
  double accW[NC][AP];
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int a = 0; a < AP; ++a) accW[j][a] = 0.0;
  double accb = 0.0, accls = 0.0;  // lane a (< A) accumulates component a
  double bzr[NC], accz[NC];         // folded bias of z and its gradient (column sums of dz)
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    bzr[j] = (bz && l + 64 * j < H) ? bz[l + 64 * j] : 0.0;
    accz[j] = 0.0;
  }
  // kPF rows in flight per wave: the z row, g (broadcast) and act / mu (lane a: component a)
  // are loaded kPF rows ahead (register ring; slots are compile-time after unrolling).
  constexpr int kPF = MEPOL_HEAD_BWD_PF;
  struct Slot {
    double z[NC];
    double g, av, mv;
  };
  Slot ring[kPF];
  // Unconditional loads from clamped (in-bounds) addresses: no exec-mask branches around the
  // loads, so they issue back to back and stay in flight.  Values of clamped columns / rows /
  // components are never used (zero weights / bias, guarded stores, guarded rows, zeroed a >= A).
  const int64_t last = N - 1;
  // Only vector loads (g through a laundered zero lane offset, so its address stays out of
  // SGPRs): scalar loads of the prefetched row's g / act / mu shared lgkmcnt with the LDS reads
  // of Wm, so the first LDS wait of a row also waited for the next row's scalars.
  int vzero = 0;
  asm volatile("" : "+v"(vzero));
  const int la = l < A ? l : A - 1;
  auto load_slot = [&](Slot& dst, int64_t i) {
    const int64_t ic = i < N ? i : last;
    const double* zr = z + ic * H;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = l + 64 * j;
      dst.z[j] = zr[c < H ? c : H - 1];
    }
    dst.g = gl[ic + vzero];
    dst.av = act[ic * A + la];
    dst.mv = mu[ic * A + la];
  };
  auto row_step = [&](int64_t i, Slot& slot) {
    double zc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) zc[j] = slot.z[j];
    const double g = slot.g;
    // lane a < A forms dmu_a, then every lane takes dmu_0..A-1 into SGPRs (the same products in
    // the same order as when every lane formed all of them)
    const double d = (l < A) ? slot.av - slot.mv : 0.0;
    const double dml = g * d * inv;
    double dm[AP];
#pragma unroll
    for (int a = 0; a < AP; ++a) dm[a] = readlane_d(dml, a);
    accb += (l < A) ? dml : 0.0;
    accls += (l < A) ? g * (-1.0 + d * d * es3) : 0.0;
    load_slot(slot, i + kPF * nwaves);
    double* dzr = dz ? dz + i * H : nullptr;
    int lo = l;
    asm volatile("" : "+v"(lo));  // keep the Wm LDS reads in the loop (no hoist into VGPRs)
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = l + 64 * j;
      const double zb = zc[j] + bzr[j];
      const double x = fmax(zb, 0.0);
      double dh = 0.0;
#pragma unroll
      for (int a = 0; a < AP; ++a) {
        dh = fma(dm[a], sW[(j * AP + a) * 64 + lo], dh);
        accW[j][a] = fma(dm[a], x, accW[j][a]);
      }
      const double dzv = (zb > 0.0) ? dh : 0.0;
      accz[j] += dzv;
      if (dzr && c < H) dzr[c] = dzv;
    }
  };
  const int64_t wave_u = __builtin_amdgcn_readfirstlane((int)wave);
#pragma unroll
  for (int p = 0; p < kPF; ++p) load_slot(ring[p], wave_u + p * nwaves);
  for (int64_t i = wave_u; i < N; i += kPF * nwaves) {
#pragma unroll
    for (int p = 0; p < kPF; ++p)
      if (i + p * nwaves < N) row_step(i + p * nwaves, ring[p]);
  }
  // block reduction in a fixed order (waves 0..3), then one record per block
  if (l < AP) {
    sb[w][l] = accb;
    sls[w][l] = accls;
  }
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
#pragma unroll
        for (int a = 0; a < AP; ++a) {
          const int idx = (a * NC + j) * 64 + l;
          sRed[idx] = (ww == 0 ? 0.0 : sRed[idx]) + accW[j][a];
        }
    }
    __syncthreads();
  }
  // column sums of dz, same fixed wave order, in the tail of sRed
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int idx = AP * 64 * NC + j * 64 + l;
        sRed[idx] = (ww == 0 ? 0.0 : sRed[idx]) + accz[j];
      }
    }
    __syncthreads();
  }
  // partial record: [dW (A*H) | db (A) | dls (A) | dbz (H)]
  const int64_t m = (int64_t)A * H + 2 * A + H;
  double* rec = part + (int64_t)blockIdx.x * m;
  for (int e = threadIdx.x; e < A * H; e += blockDim.x) {
    const int a = e / H, c = e % H;
    const int j = c >> 6, ll = c & 63;
    const int idx = (a * NC + j) * 64 + ll;
    rec[e] = sRed[idx];
  }
  if (threadIdx.x < A) {
    const int a = threadIdx.x;
    rec[A * H + a] = ((sb[0][a] + sb[1][a]) + sb[2][a]) + sb[3][a];
    rec[A * H + A + a] = ((sls[0][a] + sls[1][a]) + sls[2][a]) + sls[3][a];
  }
  for (int c = threadIdx.x; c < H; c += blockDim.x) rec[A * H + 2 * A + c] = sRed[AP * 64 * NC + c];
}

// Backward for wide action spaces (8 < A <= 32: Humanoid 17, HandReach 20).  The per-lane dWm
// accumulators of head_bwd_kernel would be NC x A doubles (5 x 24 at H = 300: over the register
// file), so here a block of ceil(H/64) waves owns one column per lane (c = threadIdx.x) and each
// lane accumulates AP values.  kRows rows per step share each Wm read from LDS and give the FMA
// chains independent work.  dmu is lane-distributed (lane a holds component a) and broadcast with
// v_readlane; Wm sits in LDS as [a][Hs] (Hs = block width, dynamic LDS, AP * Hs doubles).  The
// block walks rows in a fixed order (grid-stride), so each block's partial record
// [dW (A*H) | db (A) | dls (A) | dbz (H)] is deterministic and reduce_partials_kernel sums the
// records in a fixed order as for head_bwd_kernel.

template <int AP>
__global__ __launch_bounds__(512) void head_bwd_wide_kernel(
    const double* __restrict__ gl, const double* __restrict__ z, int64_t N, int H, int Hs,
    const double* __restrict__ bz, const double* __restrict__ Wm, const double* __restrict__ log_std,
    const double* __restrict__ act, const double* __restrict__ mu, int A,
    double* __restrict__ dz, double* __restrict__ part) {
  constexpr int kRows = 2;
  extern __shared__ double sWd[];  // [a < AP][c < Hs], then dmu[wave][row][a < AP]
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  double2* sDm = reinterpret_cast<double2*>(sWd + AP * Hs) + w * (kRows * AP / 2);
  for (int e = tid; e < AP * Hs; e += blockDim.x) {
    const int a = e / Hs, c = e % Hs;
    sWd[e] = (a < A && c < H) ? Wm[a * H + c] : 0.0;
  }
  double inv = 0.0, es3 = 0.0;  // lane a (< A): 1/sigma_a^2, exp(ls)/sigma^3
  if (l < A) {
    const double e = exp(log_std[l]);
    const double sd = e + kStdEps;
    inv = 1.0 / (sd * sd);
    es3 = e / (sd * sd * sd);
  }
  __syncthreads();
  const int c = tid;
  const int cc = c < H ? c : H - 1;  // clamped column: loads in bounds, results discarded
  const double bzc = (bz && c < H) ? bz[c] : 0.0;
  double accW[AP];
#pragma unroll
  for (int a = 0; a < AP; ++a) accW[a] = 0.0;
  double accz = 0.0, accb = 0.0, accls = 0.0;
  const int64_t last = N - 1;
  const int la = l < A ? l : A - 1;
  struct Slot {
    double z[kRows], g[kRows], av[kRows], mv[kRows];
  };
  auto load_slot = [&](Slot& s, int64_t i) {
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int64_t ic = i + r < N ? i + r : last;
      s.z[r] = z[ic * H + cc];
      s.g[r] = gl[ic];
      s.av[r] = act[ic * A + la];
      s.mv[r] = mu[ic * A + la];
    }
  };
  const int64_t stride = (int64_t)gridDim.x * kRows;
  const int64_t i0 = (int64_t)__builtin_amdgcn_readfirstlane((int)blockIdx.x) * kRows;
  Slot cur;
  load_slot(cur, i0);
  for (int64_t i = i0; i < N; i += stride) {
    Slot s = cur;
    load_slot(cur, i + stride);
    double dm[kRows], x[kRows], zb[kRows], dh[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const bool rowv = i + r < N;
      const double d = (l < A && rowv) ? s.av[r] - s.mv[r] : 0.0;
      dm[r] = s.g[r] * d * inv;  // 0 for lanes >= A and rows past N
      if (l < A && rowv) {
        accb += dm[r];
        accls += s.g[r] * (-1.0 + d * d * es3);
      }
      zb[r] = s.z[r] + bzc;
      x[r] = rowv ? fmax(zb[r], 0.0) : 0.0;
      dh[r] = 0.0;
    }
    // broadcast dmu through this wave's LDS slot (one wave's LDS ops complete in order):
    // lane a writes component a, every lane reads pairs with ds_read_b128
    if (l < AP) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) reinterpret_cast<double*>(sDm)[r * AP + l] = dm[r];
    }
    int cl = c;
    asm volatile("" : "+v"(cl));  // keep the Wm LDS reads in the loop
#pragma unroll
    for (int a2 = 0; a2 < AP / 2; ++a2) {
      const double w0 = sWd[(2 * a2) * Hs + cl];
      const double w1 = sWd[(2 * a2 + 1) * Hs + cl];
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        const double2 sa = sDm[r * (AP / 2) + a2];
        dh[r] = fma(sa.x, w0, dh[r]);
        dh[r] = fma(sa.y, w1, dh[r]);
        accW[2 * a2] = fma(sa.x, x[r], accW[2 * a2]);
        accW[2 * a2 + 1] = fma(sa.y, x[r], accW[2 * a2 + 1]);
      }
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const double dzv = (zb[r] > 0.0) ? dh[r] : 0.0;
      if (i + r < N) {
        accz += dzv;
        if (dz && c < H) dz[(i + r) * H + c] = dzv;
      }
    }
  }
  const int64_t m = (int64_t)A * H + 2 * A + H;
  double* rec = part + (int64_t)blockIdx.x * m;
  if (c < H) {
#pragma unroll
    for (int a = 0; a < AP; ++a)
      if (a < A) rec[a * H + c] = accW[a];
    rec[A * H + 2 * A + c] = accz;
  }
  // db / dlog_std: every wave accumulated the same rows' components; wave 0 writes
  if (w == 0 && l < A) {
    rec[A * H + l] = accb;
    rec[A * H + A + l] = accls;
  }
}

// out = sum_b part[b][:] in a fixed order: 64 elements per block, wave w sums a quarter of the
// partials, the 4 quarter sums are added in order.  dW goes to dWm, the tail to dbm / dls.
// Sum of the per-block partial records in two fixed-order stages (one block column per 64
// elements with all records serial per wave was latency-bound, 35 us at C3): stage 1 sums
// record group g (kRedGroups strided groups) for 64 elements per block, stage 2 sums the groups
// in order and scatters into dWm | dbm | dls | dbz.
constexpr int kRedGroups = 8;

__global__ __launch_bounds__(256) void reduce_partials_kernel(const double* __restrict__ part,
                                                              int nblocks, int64_t m,
                                                              double* __restrict__ grp) {
  __shared__ double sh[4][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + l;
  const int gi = blockIdx.y;
  double s = 0.0;
  if (e < m)
    for (int b = gi + kRedGroups * w; b < nblocks; b += 4 * kRedGroups)
      s += part[(int64_t)b * m + e];
  sh[w][l] = s;
  __syncthreads();
  if (w == 0 && e < m) grp[(int64_t)gi * m + e] = ((sh[0][l] + sh[1][l]) + sh[2][l]) + sh[3][l];
}

__global__ __launch_bounds__(256) void reduce_groups_kernel(const double* __restrict__ grp,
                                                            int64_t m, int AH, int A,
                                                            double* __restrict__ dWm,
                                                            double* __restrict__ dbm,
                                                            double* __restrict__ dls,
                                                            double* __restrict__ dbz) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  double t = 0.0;
#pragma unroll
  for (int g = 0; g < kRedGroups; ++g) t += grp[(int64_t)g * m + e];
  if (e < AH)
    dWm[e] = t;
  else if (e < AH + A)
    dbm[e - AH] = t;
  else if (e < AH + 2 * A)
    dls[e - AH - A] = t;
  else if (dbz)
    dbz[e - AH - 2 * A] = t;
}

static int reduce_records(const double* part, int nb, int64_t m, int AH, int A, double* dWm,
                          double* dbm, double* dls, double* dbz, hipStream_t st) {
  double* grp = const_cast<double*>(part) + (size_t)nb * m;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((unsigned)((m + 63) / 64), kRedGroups),
                     dim3(256), 0, st, part, nb, m, grp);
  MEPOL_CHECK_LAUNCH();
  hipLaunchKernelGGL(reduce_groups_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st,
                     grp, m, AH, A, dWm, dbm, dls, dbz);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

#ifndef MEPOL_HEAD_BWD_MAXB
#define MEPOL_HEAD_BWD_MAXB 512  // head_bwd_kernel blocks (partial records) at most
#endif
static int grid_bwd(int64_t N) {
  const int64_t waves = (N + 31) / 32;  // >= 32 rows per wave
  return (int)std::max<int64_t>(1, std::min<int64_t>(MEPOL_HEAD_BWD_MAXB, (waves + 3) / 4));
}

}  // namespace head
}  // namespace mepol

using namespace mepol;
using namespace mepol::head;

extern "C" int mepol_head_forward(const double* z, int64_t n, int hidden, const double* bz,
                                  const double* Wm, const double* bm, const double* log_std,
                                  const double* act, int a_dim, double* mu_out, double* logp_out,
                                  void* stream) {
  if (n < 0 || hidden <= 0 || hidden > 64 * kMaxCols || a_dim <= 0 || a_dim > kMaxA || !z ||
      !Wm || !bm || !log_std || !act || !mu_out || !logp_out) {
    set_error("mepol_head_forward: bad arguments (hidden <= 512, action_dim <= 32)");
    return kErrBadArg;
  }
  if (n == 0) return 0;
  const int ap = a_dim <= 1 ? 1 : a_dim <= 2 ? 2 : a_dim <= 4 ? 4 : 8;
  const int nch = (a_dim + 7) / 8;  // chunks of 8 actions (a_dim > 8)
  const int ncl16 = (hidden + 15) / 16;
  const int ncl = ncl16 <= 4 ? 4 : ncl16 <= 8 ? 8 : ncl16 <= 12 ? 12 : ncl16 <= 16 ? 16
                : ncl16 <= 20 ? 20 : ncl16 <= 24 ? 24 : 32;
  const int64_t groups = (n + 3) / 4;
  dim3 g((unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, (groups / 4 + 3) / 4)));
  hipStream_t st = (hipStream_t)stream;
#define MEPOL_HEAD_FWD(AP_, NC_, NCH_)                                                       \
  if (ap == AP_ && ncl == NC_ && nch == NCH_)                                                \
    hipLaunchKernelGGL((head_fwd16_kernel<AP_, NC_, NCH_>), g, dim3(256), 0, st, z, n, hidden, \
                       bz, Wm, bm, log_std, act, a_dim, mu_out, logp_out);
#define MEPOL_HEAD_FWD_A(AP_, NCH_)                                                    \
  MEPOL_HEAD_FWD(AP_, 4, NCH_) MEPOL_HEAD_FWD(AP_, 8, NCH_) MEPOL_HEAD_FWD(AP_, 12, NCH_) \
  MEPOL_HEAD_FWD(AP_, 16, NCH_) MEPOL_HEAD_FWD(AP_, 20, NCH_) MEPOL_HEAD_FWD(AP_, 24, NCH_) \
  MEPOL_HEAD_FWD(AP_, 32, NCH_)
  MEPOL_HEAD_FWD_A(1, 1) MEPOL_HEAD_FWD_A(2, 1) MEPOL_HEAD_FWD_A(4, 1) MEPOL_HEAD_FWD_A(8, 1)
  MEPOL_HEAD_FWD_A(8, 2) MEPOL_HEAD_FWD_A(8, 3) MEPOL_HEAD_FWD_A(8, 4)
#undef MEPOL_HEAD_FWD_A
#undef MEPOL_HEAD_FWD
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_head_workspace_size(int64_t n, int hidden, int a_dim, size_t* bytes) {
  if (!bytes || hidden <= 0 || a_dim <= 0) return kErrBadArg;
  const int nb = grid_bwd(std::max<int64_t>(n, 1));
  *bytes = ((size_t)nb + kRedGroups) * ((size_t)a_dim * (hidden + 2) + hidden) * sizeof(double);
  return 0;
}

// dz [n, hidden] (nullable: skip the input gradient), dWm [a_dim, hidden], dbm [a_dim],
// dlog_std [a_dim] are written (not accumulated).
// phase 0: the whole backward; 1: the row kernel only (its per-block records into the
// workspace, and dz); 2: the two fixed-order reduces of those records only (dWm, dbm,
// dlog_std, dbz), e.g. on another stream ordered after phase 1.
static int head_backward(const double* grad_logp, const double* z, int64_t n, int hidden,
                         const double* bz, const double* Wm, const double* log_std,
                         const double* act, const double* mu, int a_dim, double* dz, double* dWm,
                         double* dbm, double* dlog_std, double* dbz, void* workspace,
                         size_t workspace_bytes, int phase, void* stream) {
  if (n <= 0 || hidden <= 0 || hidden > 64 * kMaxCols || a_dim <= 0 || a_dim > kMaxA ||
      !grad_logp || !z || !Wm || !log_std || !act || !mu || !dWm || !dbm || !dlog_std ||
      !workspace) {
    set_error("mepol_head_backward: bad arguments");
    return kErrBadArg;
  }
  const int nb = grid_bwd(n);
  const size_t need =
      ((size_t)nb + kRedGroups) * ((size_t)a_dim * (hidden + 2) + hidden) * sizeof(double);
  if (workspace_bytes < need) {
    set_error("mepol_head_backward: workspace %zu < %zu", workspace_bytes, need);
    return kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  double* pdW = (double*)workspace;
  const int64_t m = (int64_t)a_dim * hidden + 2 * a_dim + hidden;
  if (phase == 2) return reduce_records(pdW, nb, m, a_dim * hidden, a_dim, dWm, dbm, dlog_std, dbz, st);
  if (a_dim > 8) {
    const int apw = a_dim <= 12 ? 12 : a_dim <= 16 ? 16 : a_dim <= 20 ? 20 : a_dim <= 24 ? 24 : 32;
    const int hs = (hidden + 63) / 64 * 64;  // block width: one column per lane
    const size_t lds = ((size_t)apw * hs + (size_t)(hs / 64) * 2 * apw) * sizeof(double);
#define MEPOL_HEAD_BWDW(AP_)                                                                    \
  if (apw == AP_) {                                                                             \
    static bool attr_set = false;                                                               \
    if (!attr_set) {                                                                            \
      MEPOL_HIP(hipFuncSetAttribute((const void*)head_bwd_wide_kernel<AP_>,                     \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));   \
      attr_set = true;                                                                          \
    }                                                                                           \
    hipLaunchKernelGGL((head_bwd_wide_kernel<AP_>), dim3(nb), dim3(hs), lds, st, grad_logp, z, n, \
                       hidden, hs, bz, Wm, log_std, act, mu, a_dim, dz, pdW);                   \
  }
    MEPOL_HEAD_BWDW(12) MEPOL_HEAD_BWDW(16) MEPOL_HEAD_BWDW(20) MEPOL_HEAD_BWDW(24)
    MEPOL_HEAD_BWDW(32)
#undef MEPOL_HEAD_BWDW
    MEPOL_CHECK_LAUNCH();
    if (phase == 1) return 0;
    return reduce_records(pdW, nb, m, a_dim * hidden, a_dim, dWm, dbm, dlog_std, dbz, st);
  }
  const int nc = (hidden + 63) / 64;
  const int ap = a_dim <= 1 ? 1 : a_dim <= 2 ? 2 : a_dim <= 4 ? 4 : 8;
  dim3 g(nb);
#define MEPOL_HEAD_BWD(AP_, NC_)                                                                  \
  if (ap == AP_ && nc == NC_)                                                                     \
    hipLaunchKernelGGL((head_bwd_kernel<AP_, NC_>), g, dim3(256), 0, st, grad_logp, z, n, hidden, \
                       bz, Wm, log_std, act, mu, a_dim, dz, pdW);
#define MEPOL_HEAD_BWD_A(AP_) \
  MEPOL_HEAD_BWD(AP_, 1) MEPOL_HEAD_BWD(AP_, 2) MEPOL_HEAD_BWD(AP_, 3) MEPOL_HEAD_BWD(AP_, 4) \
  MEPOL_HEAD_BWD(AP_, 5) MEPOL_HEAD_BWD(AP_, 6) MEPOL_HEAD_BWD(AP_, 7) MEPOL_HEAD_BWD(AP_, 8)
  MEPOL_HEAD_BWD_A(1) MEPOL_HEAD_BWD_A(2) MEPOL_HEAD_BWD_A(4) MEPOL_HEAD_BWD_A(8)
#undef MEPOL_HEAD_BWD_A
#undef MEPOL_HEAD_BWD
  MEPOL_CHECK_LAUNCH();
  if (phase == 1) return 0;
  return reduce_records(pdW, nb, m, a_dim * hidden, a_dim, dWm, dbm, dlog_std, dbz, st);
}

extern "C" int mepol_head_backward(const double* grad_logp, const double* z, int64_t n, int hidden,
                                   const double* bz, const double* Wm, const double* log_std,
                                   const double* act, const double* mu, int a_dim, double* dz,
                                   double* dWm, double* dbm, double* dlog_std, double* dbz,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  return head_backward(grad_logp, z, n, hidden, bz, Wm, log_std, act, mu, a_dim, dz, dWm, dbm,
                       dlog_std, dbz, workspace, workspace_bytes, 0, stream);
}

extern "C" int mepol_head_backward_phase(const double* grad_logp, const double* z, int64_t n,
                                         int hidden, const double* bz, const double* Wm,
                                         const double* log_std, const double* act,
                                         const double* mu, int a_dim, double* dz, double* dWm,
                                         double* dbm, double* dlog_std, double* dbz,
                                         void* workspace, size_t workspace_bytes, int phase,
                                         void* stream) {
  if (phase != 1 && phase != 2) {
    set_error("mepol_head_backward_phase: phase must be 1 (row kernel) or 2 (reduces)");
    return kErrBadArg;
  }
  return head_backward(grad_logp, z, n, hidden, bz, Wm, log_std, act, mu, a_dim, dz, dWm, dbm,
                       dlog_std, dbz, workspace, workspace_bytes, phase, stream);
}
