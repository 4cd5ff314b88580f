// All-pairs exact k-NN for the MEPOL particle batch on gfx950 (CDNA4, wave64).
//
// Replaces the sklearn call of the reference
//   nbrs = NearestNeighbors(n_neighbors=k+1, metric='euclidean', algorithm='auto')
//   nbrs.fit(next_states); distances, indices = nbrs.kneighbors(next_states)
// (src/algorithms/mepol.py:190-192).  Output contract = the pinned sklearn 0.22 kd_tree:
// distances are sqrt(sum_f (x_f - y_f)^2) evaluated in f64 over the f32 inputs, rows sorted
// ascending; ties are broken by the smaller candidate index (sklearn leaves tie order
// implementation-defined, so this is the build's documented convention).
//
// Pipeline (all on one stream, no host sync, no allocation):
//   1. pack    : candidates -> MFMA A-fragment tiles, A = [-2 c, |c|^2] (fp32), max |c|.
//   2. select  : v_mfma_f32_32x32x2_f32 computes |c|^2 - 2 q.c for 32 candidates x 32 queries
//                per 15-MFMA step (d = 29); each lane owns one query column and keeps a
//                sorted top-LIST list in VGPRs, fed through a per-lane LDS buffer so the
//                wave pays the insertion cost in batches, not per candidate.
//   3. refine  : per query, merge the 2*split partial lists to the approximate top-LIST,
//                recompute those distances exactly in f64, bitonic-sort by (dist, idx), and
//                certify with a rigorous fp32 error bound that no excluded candidate can
//                enter the top-(k+1).  Uncertified queries (near-ties across the boundary,
//                large duplicate clusters) are queued.
//   4. exact   : queued queries are answered by an exhaustive f64 scan (no approximation).
#include "common.hpp"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdlib>

namespace mepol {
namespace knn {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;

constexpr float kPadNorm = 1e30f;  // |c|^2 of padding candidates: never selected
constexpr int kBufCap = 24;        // per-lane LDS insertion buffer (entries)
constexpr int kMaxSplit = 16;

// ---------------------------------------------------------------------------------------
// 1. pack
// ---------------------------------------------------------------------------------------
// apack[(t*64 + l)*KSP + s] = A[i = l&31][k = l>>5] of k-step s for candidate tile t, i.e.
// feature f = 2s + (l>>5) of candidate c = 32t + (l&31):  f<d: -2 x_cf ; f==d: |c|^2 ; else 0.
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ X, int64_t n, int d,
                                                   int KSP, int64_t nct,
                                                   float* __restrict__ apack,
                                                   unsigned* __restrict__ cmax_bits) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = nct * 64;
  float mynorm = 0.f;
  if (gid < total) {
    const int64_t t = gid >> 6;
    const int l = (int)(gid & 63);
    const int h = l >> 5;
    const int64_t c = t * 32 + (l & 31);
    const bool valid = c < n;
    float cn = 0.f;
    if (valid) {
      const float* xc = X + c * d;
      for (int f = 0; f < d; ++f) cn = fmaf(xc[f], xc[f], cn);
    }
    float* dst = apack + gid * KSP;
    for (int s = 0; s < KSP; s += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int f = 2 * (s + u) + h;
        float x;
        if (valid)
          x = (f < d) ? -2.f * X[c * d + f] : ((f == d) ? cn : 0.f);
        else
          x = (f == d) ? kPadNorm : 0.f;
        v[u] = x;
      }
      *reinterpret_cast<float4*>(dst + s) = make_float4(v[0], v[1], v[2], v[3]);
    }
    if (valid && h == 0) mynorm = sqrtf(cn);
  }
  // wave max -> one atomic per wave (non-negative floats order like their bit patterns)
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) mynorm = fmaxf(mynorm, __shfl_xor(mynorm, m, kWave));
  if ((threadIdx.x & 63) == 0) atomicMax(cmax_bits, __float_as_uint(mynorm));
}

// ---------------------------------------------------------------------------------------
// 2. select
// ---------------------------------------------------------------------------------------
template <int LIST>
__device__ __forceinline__ void list_insert(float (&ld)[LIST], int (&li)[LIST], float x, int xi) {
  // ld ascending; precondition x < ld[LIST-1].  Branch-free shift-insert.
  bool c[LIST];
#pragma unroll
  for (int j = 0; j < LIST; ++j) c[j] = x < ld[j];
#pragma unroll
  for (int j = LIST - 1; j >= 1; --j) {
    ld[j] = c[j - 1] ? ld[j - 1] : (c[j] ? x : ld[j]);
    li[j] = c[j - 1] ? li[j - 1] : (c[j] ? xi : li[j]);
  }
  ld[0] = c[0] ? x : ld[0];
  li[0] = c[0] ? xi : li[0];
}

// Merge this lane's LDS buffer into its sorted list; then share the prune bound with the
// partner lane (l ^ 32 serves the same query column).  Every lane of the wave calls it.
// keep > 0 (split-f16 select): the bound also takes max(own keep-th, partner's keep-th): the
// two half lists then hold >= 2 keep values at or below it, so 2 keep >= kp1 + slack of the
// query's candidates in this range are never pruned; this bound is far tighter than a list's
// own last entry (the LIST-th of one half).  The bound only decreases over the scan.
template <int LIST>
__device__ __forceinline__ float list_at(const float (&ld)[LIST], int j) {
  float v = INFINITY;
#pragma unroll
  for (int i = 0; i < LIST; ++i) v = (i == j) ? ld[i] : v;
  return v;
}

template <int LIST>
__device__ __forceinline__ void flush_buffer(float (&ld)[LIST], int (&li)[LIST], float& thr, int& cnt,
                                             const float (*bv)[64], const int (*bi)[64], int l,
                                             float thr0, int keep = 0) {
  const int mc = wave_max_i(cnt);
#pragma nounroll
  for (int e = 0; e < mc; ++e) {
    if (e < cnt) {
      const float x = bv[e][l];
      const int xi = bi[e][l];
      if (x < thr) {
        list_insert<LIST>(ld, li, x, xi);
        thr = ld[LIST - 1];
      }
    }
  }
  cnt = 0;
  // lanes l and l^32 serve the same query: the tighter of their maxima is a valid prune bound
  // for both (refine's certification bound is the min over all lanes' final bounds and the
  // query's sampled bound thr0).
  thr = fminf(thr0, fminf(ld[LIST - 1], __shfl_xor(ld[LIST - 1], 32, kWave)));
  if (keep > 0) {
    const float kv = list_at<LIST>(ld, keep - 1);
    thr = fminf(thr, fmaxf(kv, __shfl_xor(kv, 32, kWave)));
  }
}

// Row (candidate within the tile) of accumulator register r for lane l (32x32 C/D map).
__device__ __forceinline__ int acc_row(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }

template <int KS, int KSP, int LIST>
__global__ __launch_bounds__(256) void select_kernel(const float* __restrict__ apack,
                                                     const float* __restrict__ query, int64_t nq,
                                                     int d, int64_t nct, int split,
                                                     int64_t tiles_per_split,
                                                     float* __restrict__ out_v,
                                                     int* __restrict__ out_i) {
  __shared__ float sbuf_v[4][kBufCap][64];
  __shared__ int sbuf_i[4][kBufCap][64];
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  const int64_t qt = (int64_t)blockIdx.x * 4 + w;
  const int sp = blockIdx.y;
  if (qt * 32 >= nq) return;  // wave-uniform
  const int h = l >> 5;
  const int64_t q = qt * 32 + (l & 31);
  const bool qvalid = q < nq;

  // B operand (queries): B[k = h][j = l&31] of step s = feature 2s + h; f == d carries 1.
  float bq[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int f = 2 * s + h;
    bq[s] = qvalid ? ((f < d) ? query[q * d + f] : ((f == d) ? 1.f : 0.f)) : 0.f;
  }

  // Retire the B-operand loads here and launder the registers, so no compiler-tracked load is
  // pending inside the tile loop (otherwise its waitcnt pass drains vmcnt(0) every iteration).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(bq[s]));

  float ld[LIST];
  int li[LIST];
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    ld[j] = INFINITY;
    li[j] = -1;
  }
  const float thr0 = INFINITY;
  float thr = thr0;
  int cnt = 0;

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  constexpr int NV = KSP / 4;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack + (int64_t)l * KSP);
  // Two register buffers (ping-pong): tile t+1's loads are in flight while tile t's MFMA chain
  // runs.  Fragment loads are issued from inline asm so the compiler's waitcnt pass (which
  // drains to vmcnt(0) at this loop's control-flow joins) does not see them; the waits are
  // counted by hand: the only vector-memory ops inside the loop are these NV loads per tile.
  f32x4 A0[NV], A1[NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 16 * KSP;  // 64 lanes * KSP floats = 16*KSP f32x4 per tile
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x;
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x) : "v"(p + v) : "memory");
      A[v] = x;
    }
  };
  auto wait_older = [&](f32x4 (&A)[NV]) {  // all but the NV youngest loads have landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV) : "memory");
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x = A[v];
      asm volatile("" : "+v"(x));
      A[v] = x;
    }
  };
  auto wait_all = [&](f32x4 (&A)[NV]) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x = A[v];
      asm volatile("" : "+v"(x));
      A[v] = x;
    }
  };
  auto comp = [](const f32x4 (&A)[NV], int s) -> float { return A[s >> 2][s & 3]; };
  auto tile = [&](const f32x4 (&A)[NV], int64_t t) {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(A, s), bq[s], acc, 0, 0, 0);
    float m = fminf(fminf(fminf(acc[0], acc[1]), fminf(acc[2], acc[3])),
                    fminf(fminf(acc[4], acc[5]), fminf(acc[6], acc[7])));
    m = fminf(m, fminf(fminf(fminf(acc[8], acc[9]), fminf(acc[10], acc[11])),
                       fminf(fminf(acc[12], acc[13]), fminf(acc[14], acc[15]))));
    if (__ballot(m < thr)) {
      const int base = (int)(t * 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (acc[r] < thr) {
          sbuf_v[w][cnt][l] = acc[r];
          sbuf_i[w][cnt][l] = base + acc_row(r, l);
          ++cnt;
        }
      }
      if (__ballot(cnt > kBufCap - 16)) flush_buffer<LIST>(ld, li, thr, cnt, sbuf_v[w], sbuf_i[w], l, thr0);
    }
  };
  if (t0 < t1) {
    load(A0, t0);
    int64_t t = t0;
#pragma nounroll
    for (; t + 1 < t1; t += 2) {
      load(A1, t + 1);
      wait_older(A0);
      tile(A0, t);
      load(A0, min(t + 2, t1 - 1));
      wait_older(A1);
      tile(A1, t + 1);
    }
    wait_all(A0);
    if (t < t1) tile(A0, t);
  }
  flush_buffer<LIST>(ld, li, thr, cnt, sbuf_v[w], sbuf_i[w], l, thr0);

  if (qvalid) {
    const int64_t o = ((q * split + sp) * 2 + h) * LIST;
#pragma unroll
    for (int j = 0; j < LIST; ++j) {
      out_v[o + j] = ld[j];
      out_i[o + j] = li[j];
    }
  }
}

// ---------------------------------------------------------------------------------------
// 2b. select on split-f16 MFMA (default): the same |c|^2 - 2 q.c, with every operand split
//     into two f16 halves, a = a_hi + a_lo (|a - a_hi - a_lo| <= 2^-22 |a|), and the three
//     products hi*hi + hi*lo + lo*hi accumulated in f32 by v_mfma_f32_32x32x16_f16 (exact
//     products, f32 sums): ~f32-class accuracy at 3 MFMAs of 16x the f32 rate.  Coordinates
//     are scaled by a power of two sigma (max norm -> (64, 128]) so |c|^2 fits f16; outputs
//     are unscaled exactly.  refine's certification uses this path's error bound.
// ---------------------------------------------------------------------------------------
// max |x| over candidates (scal[0]) and over queries (scal[2]), non-negative float bit order.
// Input validation (sklearn's check_array inside NearestNeighbors.fit / kneighbors,
// mepol.py:190-192): rows with a NaN / inf coordinate are counted in bad[0], rows whose f32
// squared norm overflows (|x| >~ 1.8e19) in bad[1].  The tests are on laundered bit patterns: this
// TU is built with -fno-honor-nans (for the selection kernels), under which the compiler rewrites
// a plain exponent test into |x| == inf and loses NaN.  Once validated, no NaN reaches the
// selection / refine / exact kernels, so the flag cannot change their results.
__device__ __forceinline__ bool nonfinite_bits(float v) {
  unsigned b = __float_as_uint(v);
  asm volatile("" : "+v"(b));
  return (b & 0x7f800000u) == 0x7f800000u;
}

__global__ __launch_bounds__(256) void norms_kernel(const float* __restrict__ X, int64_t n, int d,
                                                    unsigned* __restrict__ out_bits,
                                                    unsigned* __restrict__ bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float nrm = 0.f;
  bool nonfinite = false, overflow = false;
  if (i < n) {
    const float* x = X + i * d;
    float s2 = 0.f;
    for (int f = 0; f < d; ++f) {
      nonfinite |= nonfinite_bits(x[f]);
      s2 = fmaf(x[f], x[f], s2);
    }
    overflow = !nonfinite && nonfinite_bits(s2);
    nrm = (nonfinite || overflow) ? 0.f : sqrtf(s2);
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) nrm = fmaxf(nrm, __shfl_xor(nrm, m, kWave));
  if ((threadIdx.x & 63) == 0) atomicMax(out_bits, __float_as_uint(nrm));
  const unsigned long long b1 = __ballot(nonfinite), b2 = __ballot(overflow);
  if ((threadIdx.x & 63) == 0) {
    if (b1) atomicAdd(bad, (unsigned)__popcll(b1));
    if (b2) atomicAdd(bad + 1, (unsigned)__popcll(b2));
  }
}

// sigma = 2^e with sigma * max(cmax, qmax) in (64, 128] (1 when the data is all zero).
__device__ __forceinline__ float knn_scale(const unsigned* __restrict__ scal) {
  const float m = fmaxf(__uint_as_float(scal[0]), __uint_as_float(scal[2]));
  // slack for the f32 rounding of sqrt in norms_kernel: 127.9 instead of 128
  if (!(m > 0.f) || !(m < 3e38f)) return 1.f;
  int e;
  (void)frexpf(127.9f / m, &e);
  e = max(-100, min(100, e - 1));
  return ldexpf(1.f, e);
}

// Smallest float above v (v itself for +inf / NaN).
__device__ __forceinline__ float next_up(float v) {
  if (!(v < INFINITY)) return v;
  if (v == 0.f) return __uint_as_float(1u);
  const unsigned b = __float_as_uint(v);
  return __uint_as_float(v > 0.f ? b + 1u : b - 1u);
}

__device__ __forceinline__ void split_f16(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);  // v - hi is exact in f32
}

constexpr float kPadNorm16 = 60000.f;  // scaled |c|^2 of padding candidates (> any real D')

// apack16[((t*64 + l)*KS16 + s)*16 + {0..7 hi, 8..15 lo}] = A[i = l&31][k = 16 s + 8 (l>>5) + j]
// of candidate tile t: f<d: -2 sigma x_cf ; f==d: |sigma c|^2 ; else 0.
__global__ __launch_bounds__(256) void pack16_kernel(const float* __restrict__ X, int64_t n, int d,
                                                     int KS16, int64_t nct,
                                                     _Float16* __restrict__ apack,
                                                     const unsigned* __restrict__ scal) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= nct * 64) return;
  const float sg = knn_scale(scal);
  const int64_t t = gid >> 6;
  const int l = (int)(gid & 63);
  const int h = l >> 5;
  const int64_t c = t * 32 + (l & 31);
  const bool valid = c < n;
  float cn = 0.f;
  if (valid) {
    const float* xc = X + c * d;
    for (int f = 0; f < d; ++f) {
      const float y = sg * xc[f];
      cn = fmaf(y, y, cn);
    }
  }
  _Float16* dst = apack + gid * KS16 * 16;
  for (int s = 0; s < KS16; ++s) {
    f16x8 hv, lv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * s + 8 * h + j;
      float v;
      if (valid)
        v = (f < d) ? -2.f * sg * X[c * d + f] : ((f == d) ? cn : 0.f);
      else
        v = (f == d) ? kPadNorm16 : 0.f;
      _Float16 a, b;
      split_f16(v, a, b);
      hv[j] = a;
      lv[j] = b;
    }
    *reinterpret_cast<f16x8*>(dst + s * 16) = hv;
    *reinterpret_cast<f16x8*>(dst + s * 16 + 8) = lv;
  }
}

// TAU = false: partial top-LIST lists of every query over its split's tile range, pruned from the
//              start by the query's sampled bound tau_in (scaled units; nullptr = none).
// TAU = true : the sampling pass.  Tiles t*tile_stride (t < nct) only, split = 1; writes
//              tau_out[q] = the next float above min over the two half-lists of their kp1-th
//              value: an upper bound on the query's (k+1)-th smallest approximate value over all
//              candidates (a subset's (k+1)-th is never below the full set's), at least kp1
//              sampled candidates lie at or below it, and the values are bitwise those of the
//              main pass (same fragments, same MFMA chain).
template <int KS16, int LIST, bool TAU>
__global__ __launch_bounds__(256) void select16_kernel(const _Float16* __restrict__ apack,
                                                       const float* __restrict__ query,
                                                       int64_t nq, int d, int64_t nct, int split,
                                                       int64_t tiles_per_split, int tile_stride,
                                                       int kp1, int keep,
                                                       const unsigned* __restrict__ scal,
                                                       const float* __restrict__ tau_in,
                                                       float* __restrict__ tau_out,
                                                       float* __restrict__ out_v,
                                                       int* __restrict__ out_i) {
  __shared__ float sbuf_v[4][kBufCap][64];
  __shared__ int sbuf_i[4][kBufCap][64];
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  if (TAU) keep = 0;
  // XCD-aware block mapping: workgroups go round-robin over the 8 XCDs by linear id, so with
  // sp = id % split (split a multiple of 8) every XCD only ever reads the candidate ranges
  // sp = xcd (mod 8), which then stay resident in that XCD's 4 MB L2 instead of streaming from
  // the Infinity Cache once per query tile.  Any other split (3 at C3) keeps the split-major
  // order: the blocks in flight then all read one candidate range, not every range at once
  // (the XCD mapping with split = 3 put all three ranges in every L2: 2.7x the fetch bytes).
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const bool xcd_map = (split & 7) == 0;
  const int sp = xcd_map ? (int)(lin % split) : (int)blockIdx.y;
  const int64_t qt = (xcd_map ? lin / split : (int64_t)blockIdx.x) * 4 + w;
  if (qt * 32 >= nq) return;  // wave-uniform
  const int h = l >> 5;
  const int64_t q = qt * 32 + (l & 31);
  const bool qvalid = q < nq;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);  // exact: sigma is a power of two

  // B operand (queries): B[k = 16 s + 8h + j][col = l&31] = sigma q_f (f<d), 1 (f==d), 0.
  f16x8 bhi[KS16], blo[KS16];
#pragma unroll
  for (int s = 0; s < KS16; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * s + 8 * h + j;
      const float v = qvalid ? ((f < d) ? sg * query[q * d + f] : ((f == d) ? 1.f : 0.f)) : 0.f;
      _Float16 a, b;
      split_f16(v, a, b);
      bhi[s][j] = a;
      blo[s][j] = b;
    }
  float thr0 = (!TAU && tau_in && qvalid) ? tau_in[q] : INFINITY;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < KS16; ++s) {
    f32x4 x = __builtin_bit_cast(f32x4, bhi[s]);
    f32x4 y = __builtin_bit_cast(f32x4, blo[s]);
    asm volatile("" : "+v"(x), "+v"(y));
    bhi[s] = __builtin_bit_cast(f16x8, x);
    blo[s] = __builtin_bit_cast(f16x8, y);
  }
  asm volatile("" : "+v"(thr0));  // retired above (see filter16_kernel)

  float ld[LIST];
  int li[LIST];
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    ld[j] = INFINITY;
    li[j] = -1;
  }
  float thr = thr0;
  int cnt = 0;

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  // Three fragment buffers: tile t's MFMAs run while tile t-1's threshold work executes and
  // tile t+1's loads are in flight; a buffer is refilled (tile t+2) only after the chain that
  // read it has completed (its results were consumed).  Loads are inline asm with hand-counted
  // waits (NV per tile; no other vector-memory op in the loop).
  constexpr int NV = 2 * KS16;  // dwordx4 per lane per tile: hi and lo halves of each k-step
  // Fragment buffers: three for KS16 <= 3; two for KS16 = 4 (d + 1 <= 64, HandReach), whose
  // 8-register-per-k-step buffers would otherwise put the kernel at the 256-VGPR cap.
  constexpr int NB = KS16 >= 4 ? 2 : 3;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + (int64_t)l * NV;
  f32x4 Bf[NB][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * tile_stride * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x;
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x) : "v"(p + v) : "memory");
      A[v] = x;
    }
  };
  auto landed = [&](f32x4 (&A)[NV]) {  // all but the NV youngest loads (next tile) have landed
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV) : "memory");
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x = A[v];
      asm volatile("" : "+v"(x));
      A[v] = x;
    }
  };
  auto chain = [&](const f32x4 (&A)[NV]) -> f32x16 {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KS16; ++s) {
      const f16x8 ah = __builtin_bit_cast(f16x8, A[2 * s]);
      const f16x8 al = __builtin_bit_cast(f16x8, A[2 * s + 1]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhi[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blo[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhi[s], acc, 0, 0, 0);
    }
    return acc;
  };
  auto process = [&](f32x16 acc, int64_t t) {
    float m = fminf(fminf(fminf(acc[0], acc[1]), fminf(acc[2], acc[3])),
                    fminf(fminf(acc[4], acc[5]), fminf(acc[6], acc[7])));
    m = fminf(m, fminf(fminf(fminf(acc[8], acc[9]), fminf(acc[10], acc[11])),
                       fminf(fminf(acc[12], acc[13]), fminf(acc[14], acc[15]))));
    if (__ballot(m < thr)) {
      const int base = (int)(t * tile_stride * 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (acc[r] < thr) {
          sbuf_v[w][cnt][l] = acc[r];
          sbuf_i[w][cnt][l] = base + acc_row(r, l);
          ++cnt;
        }
      }
      if (__ballot(cnt > kBufCap - 16))
        flush_buffer<LIST>(ld, li, thr, cnt, sbuf_v[w], sbuf_i[w], l, thr0, keep);
    }
  };
  if constexpr (NB == 2) {
    if (t0 < t1) {
      // Double buffer: tile t+1's loads are issued right after tile t's MFMA chain (the chain
      // of t-1, the last reader of that buffer, executed before chain t in the matrix pipe)
      // and land while the chain and the threshold work of t-1 run; each step then waits for
      // all outstanding loads, which are exactly tile t's.
      const int64_t tl = t1 - 1;
      load(Bf[0], t0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int v = 0; v < NV; ++v) asm volatile("" : "+v"(Bf[0][v]));
      f32x16 accP = chain(Bf[0]);
      load(Bf[1], min(t0 + 1, tl));
      int64_t t = t0 + 1;
#define MEPOL_SEL16_STEP2(CUR, NXT)                            \
  {                                                           \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          \
    _Pragma("unroll") for (int v = 0; v < NV; ++v)            \
        asm volatile("" : "+v"(Bf[CUR][v]));                  \
    const f32x16 accN = chain(Bf[CUR]);                       \
    load(Bf[NXT], min(t + 1, tl));                            \
    process(accP, t - 1);                                     \
    accP = accN;                                              \
    ++t;                                                      \
  }
#pragma nounroll
      while (t + 1 < t1) {
        MEPOL_SEL16_STEP2(1, 0)
        MEPOL_SEL16_STEP2(0, 1)
      }
      if (t < t1) MEPOL_SEL16_STEP2(1, 0)
#undef MEPOL_SEL16_STEP2
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int v = 0; v < NV; ++v) asm volatile("" : "+v"(Bf[b][v]));
      process(accP, t - 1);
    }
  } else if (t0 < t1) {
    const int64_t tl = t1 - 1;
    load(Bf[0], t0);
    load(Bf[1], min(t0 + 1, tl));
    landed(Bf[0]);
    f32x16 accP = chain(Bf[0]);
    load(Bf[2], min(t0 + 2, tl));
    int64_t t = t0 + 1;
    // steady state, unrolled by 3 so buffer indices are compile-time: at step t the tile is in
    // Bf[(t - t0) % 3], the chain of t-1 read Bf[(t - t0 - 1) % 3] (refilled with t+2).
#define MEPOL_SEL16_STEP(CUR, PREV)         \
  {                                         \
    landed(Bf[CUR]);                        \
    const f32x16 accN = chain(Bf[CUR]);     \
    process(accP, t - 1);                   \
    load(Bf[PREV], min(t + 2, tl));         \
    accP = accN;                            \
    ++t;                                    \
  }
#pragma nounroll
    while (t + 2 < t1) {
      MEPOL_SEL16_STEP(1, 0)
      MEPOL_SEL16_STEP(2, 1)
      MEPOL_SEL16_STEP(0, 2)
    }
    // remainder (0..2 tiles), same buffer rotation
    if (t < t1) MEPOL_SEL16_STEP(1, 0)
    if (t < t1) MEPOL_SEL16_STEP(2, 1)
#undef MEPOL_SEL16_STEP
    // Retire every outstanding fragment load and keep all three buffers live up to here: the
    // last prefetches are never consumed, and an asm load whose output the compiler thinks is
    // dead may be given registers that a later instruction reuses while the data is in flight.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
      for (int v = 0; v < NV; ++v) asm volatile("" : "+v"(Bf[b][v]));
    process(accP, t - 1);
  }
  flush_buffer<LIST>(ld, li, thr, cnt, sbuf_v[w], sbuf_i[w], l, thr0, keep);

  if (TAU) {
    // each half keeps its m = ceil(kp1/2) smallest; the union then holds 2m >= kp1 sampled
    // values <= max of the two m-th values, a bound about as tight as the union's kp1-th
    const int m = (kp1 + 1) / 2;
    float v = INFINITY;
#pragma unroll
    for (int j = 0; j < LIST; ++j) v = (j == m - 1) ? ld[j] : v;
    v = fmaxf(v, __shfl_xor(v, 32, kWave));
    if (qvalid && h == 0) tau_out[q] = next_up(v);
    return;
  }
  if (qvalid) {
    // The last slot carries this lane's final bound: every candidate of its range that is not
    // in the list has an approximate value >= min(list last, thr) (rejected against thr, or
    // evicted from the list); a last entry at or above the bound is dropped (idx -1), the
    // bound covers it.  refine takes the min over the query's lanes.
    const float bound = fminf(ld[LIST - 1], thr);
    const int64_t o = ((q * split + sp) * 2 + h) * LIST;
#pragma unroll
    for (int j = 0; j < LIST - 1; ++j) {
      out_v[o + j] = ld[j] * inv_s2;
      out_i[o + j] = li[j];
    }
    out_v[o + LIST - 1] = bound * inv_s2;
    out_i[o + LIST - 1] = (bound < ld[LIST - 1]) ? -1 : li[LIST - 1];
  }
}

// 2c. filter pass (split-f16, seeded by the sampling pass): no sorted lists at all.  Every
//     candidate whose approximate value is below the query's sampled bound tau (scaled units) is
//     appended to a per-lane LDS buffer; full buffers are spilled to the query's survivor array
//     (capacity cap, global count per query; entries past cap only raise the count, which makes
//     refine queue the query for the exhaustive path).  The tile loop is MFMA chain + min tree +
//     one compare per tile; with no lists in registers the accumulators stay in VGPRs.
template <int KS16>
__global__ __launch_bounds__(256) void filter16_kernel(const _Float16* __restrict__ apack,
                                                       const float* __restrict__ query,
                                                       int64_t nq, int d, int64_t nct, int split,
                                                       int64_t tiles_per_split,
                                                       const unsigned* __restrict__ scal,
                                                       const float* __restrict__ tau, int cap,
                                                       int* __restrict__ counts,
                                                       float* __restrict__ sv,
                                                       int* __restrict__ si) {
  __shared__ float sbuf_v[4][kBufCap][64];
  __shared__ int sbuf_i[4][kBufCap][64];
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  // XCD-aware block mapping (see select16_kernel)
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const int sp = (int)(lin % split);
  const int64_t qt = (lin / split) * 4 + w;
  if (qt * 32 >= nq) return;  // wave-uniform
  const int h = l >> 5;
  const int64_t q = qt * 32 + (l & 31);
  const bool qvalid = q < nq;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);

  f16x8 bhi[KS16], blo[KS16];
#pragma unroll
  for (int s = 0; s < KS16; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * s + 8 * h + j;
      const float v = qvalid ? ((f < d) ? sg * query[q * d + f] : ((f == d) ? 1.f : 0.f)) : 0.f;
      _Float16 a, b;
      split_f16(v, a, b);
      bhi[s][j] = a;
      blo[s][j] = b;
    }
  float thr = qvalid ? tau[q] : -INFINITY;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < KS16; ++s) {
    f32x4 x = __builtin_bit_cast(f32x4, bhi[s]);
    f32x4 y = __builtin_bit_cast(f32x4, blo[s]);
    asm volatile("" : "+v"(x), "+v"(y));
    bhi[s] = __builtin_bit_cast(f16x8, x);
    blo[s] = __builtin_bit_cast(f16x8, y);
  }
  // retired by the wait above: no compiler-tracked load may reach the loop (it would drain
  // vmcnt(0) at the first use in every iteration and serialise the fragment pipeline)
  asm volatile("" : "+v"(thr));
  int cnt = 0;
  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  constexpr int NV = 2 * KS16;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + (int64_t)l * NV;
  f32x4 Bf[3][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x;
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x) : "v"(p + v) : "memory");
      A[v] = x;
    }
  };
  auto landed = [&](f32x4 (&A)[NV]) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV) : "memory");
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x = A[v];
      asm volatile("" : "+v"(x));
      A[v] = x;
    }
  };
  auto chain = [&](const f32x4 (&A)[NV]) -> f32x16 {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KS16; ++s) {
      const f16x8 ah = __builtin_bit_cast(f16x8, A[2 * s]);
      const f16x8 al = __builtin_bit_cast(f16x8, A[2 * s + 1]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhi[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blo[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhi[s], acc, 0, 0, 0);
    }
    return acc;
  };
  // Spill this lane's buffer to the query's survivor array.  The returning atomic makes the
  // compiler drain vmcnt, which also retires the in-flight fragment loads (correct, and rare).
  auto spill = [&]() {
    if (cnt > 0) {
      const int base = atomicAdd(counts + q, cnt);
      for (int e = 0; e < cnt; ++e) {
        const int pos = base + e;
        if (pos < cap) {
          sv[q * cap + pos] = sbuf_v[w][e][l] * inv_s2;
          si[q * cap + pos] = sbuf_i[w][e][l];
        }
      }
    }
    cnt = 0;
    // vmcnt(0) here, visible to the compiler: its stores are complete on this rare path, so
    // the loop latch needs no drain of its own (which would serialise every tile's loads)
    __builtin_amdgcn_s_waitcnt(0x0F70);
  };
  auto process = [&](f32x16 acc, int64_t t) {
    const float m = fminf(
        fminf(fminf(fminf(acc[0], acc[1]), fminf(acc[2], acc[3])),
              fminf(fminf(acc[4], acc[5]), fminf(acc[6], acc[7]))),
        fminf(fminf(fminf(acc[8], acc[9]), fminf(acc[10], acc[11])),
              fminf(fminf(acc[12], acc[13]), fminf(acc[14], acc[15]))));
    if (__ballot(m < thr)) {
      const int base = (int)(t * 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (acc[r] < thr) {
          sbuf_v[w][cnt][l] = acc[r];
          sbuf_i[w][cnt][l] = base + acc_row(r, l);
          ++cnt;
        }
      }
      if (__ballot(cnt > kBufCap - 16)) spill();
    }
  };
  if (t0 < t1) {
    const int64_t tl = t1 - 1;
    load(Bf[0], t0);
    load(Bf[1], min(t0 + 1, tl));
    landed(Bf[0]);
    f32x16 accP = chain(Bf[0]);
    load(Bf[2], min(t0 + 2, tl));
    int64_t t = t0 + 1;
#define MEPOL_FLT16_STEP(CUR, PREV)         \
  {                                         \
    landed(Bf[CUR]);                        \
    const f32x16 accN = chain(Bf[CUR]);     \
    process(accP, t - 1);                   \
    load(Bf[PREV], min(t + 2, tl));         \
    accP = accN;                            \
    ++t;                                    \
  }
#pragma nounroll
    while (t + 2 < t1) {
      MEPOL_FLT16_STEP(1, 0)
      MEPOL_FLT16_STEP(2, 1)
      MEPOL_FLT16_STEP(0, 2)
    }
    if (t < t1) MEPOL_FLT16_STEP(1, 0)
    if (t < t1) MEPOL_FLT16_STEP(2, 1)
#undef MEPOL_FLT16_STEP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
      for (int v = 0; v < NV; ++v) asm volatile("" : "+v"(Bf[b][v]));
    process(accP, t - 1);
  }
  spill();
}

// ---------------------------------------------------------------------------------------
// 3. refine + certify
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool lex_less(double a, int ai, double b, int bi) {
  return a < b || (a == b && ai < bi);
}
__device__ __forceinline__ bool lex_less_f(float a, int ai, float b, int bi) {
  return a < b || (a == b && ai < bi);
}

// Exact f64 squared distance, summed in feature order with no contraction (matches the
// reference's kd_tree rdist: sum of (x_f - y_f)^2 in double, f = 0..d-1).
// The row is read 32 features at a time with every load issued before the first use (clamped,
// unconditional addresses): one memory latency per chunk instead of one per feature (the
// refine's random candidate rows miss L2, and the per-feature loop serialised those misses).
__device__ __forceinline__ double exact_d2(const float* __restrict__ a, const float* __restrict__ b, int d) {
  constexpr int kCh = 32;
  double s = 0.0;
  for (int f0 = 0; f0 < d; f0 += kCh) {
    float av[kCh], bv[kCh];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      const int f = min(f0 + u, d - 1);
      av[u] = a[f];
      bv[u] = b[f];
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      if (f0 + u < d) {  // uniform condition
        const double t = __dsub_rn((double)av[u], (double)bv[u]);
        s = __dadd_rn(s, __dmul_rn(t, t));
      }
    }
  }
  return s;
}

// Correctly rounded f64 square root (round-to-nearest-even, as glibc / numpy / sklearn).
// y0 = sqrt(x) is within 1 ulp; with Y = y/ulp(y) an integer, x/ulp^2 is an integer, so
// "RN(sqrt x) >= y+"  <=>  x > y*y+  and  "RN(sqrt x) <= y-"  <=>  x <= y-*y; both signs are
// exact through one fma (a rounded nonzero keeps its sign).
__device__ __forceinline__ double sqrt_rn(double x) {
  const double y = sqrt(x);
  if (!(x > 1e-290) || !(x < 1e300)) return y;
  const double yp = __longlong_as_double(__double_as_longlong(y) + 1);
  if (__builtin_fma(-y, yp, x) > 0.0) return yp;
  const double ym = __longlong_as_double(__double_as_longlong(y) - 1);
  if (__builtin_fma(-ym, y, x) <= 0.0) return ym;
  return y;
}

template <int LIST, int MAXP>
__global__ __launch_bounds__(256) void refine_kernel(
    const float* __restrict__ cand, int64_t nc, const float* __restrict__ query, int64_t nq, int d,
    int kp1, int M, int list_len, const int* __restrict__ counts,
    const float* __restrict__ lists_v, const int* __restrict__ lists_i,
    const unsigned* __restrict__ cmax_bits, int e_terms, const float* __restrict__ tau,
    double* __restrict__ Dout,
    int64_t* __restrict__ I64, int32_t* __restrict__ I32, int* __restrict__ flag_count,
    int* __restrict__ flag_list, int rank_merge) {
  __shared__ int sel[4][64];
  __shared__ float selv[4][64];  // rank merge: approximate value of sel[r]
  constexpr int kRM = MAXP <= 4 ? MAXP : 1;  // rank merge for M <= 256 entries
  __shared__ float2 sent[4][64 * kRM];        // rank merge: the query's entries (value, index bits)
  if (MAXP > 4) rank_merge = 0;
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs, so block b runs on
  // XCD b % 8; each XCD gets one contiguous range of query blocks.  Neighbouring queries' rows of
  // the transposed index table (I32[l][q], 4 bytes per query) then meet in one L2 and leave it
  // as whole lines instead of 16-byte pieces from 8 different L2s.
  const int64_t nb = gridDim.x, bx = blockIdx.x;
  const int64_t xcd = bx & 7, per = nb >> 3, rem = nb & 7;
  const int64_t qb = xcd * per + min(xcd, rem) + (bx >> 3);
  const int64_t q = qb * 4 + w;
  if (q >= nq) return;
  // Candidate entries of this query: M per query.  Lists mode (counts == nullptr): 2*split
  // ascending partial lists of list_len each.  Survivor mode: counts[q] unsorted entries (a count
  // above M means entries were dropped: the query is not certified).
  const float* lv = lists_v + q * M;
  const int* lix = lists_i + q * M;
  const int nval = counts ? min(counts[q], M) : M;
  const bool overflow = counts && counts[q] > M;

  // Bound part 1: min over partial lists of their maxima (last, lists are ascending) and the
  // sampled bound the selection started from (scaled units -> unscaled, exact power of two).
  float bnd = INFINITY;
  if (tau) {
    const float sg = knn_scale(cmax_bits);
    bnd = tau[q] / (sg * sg);
  }
  if (list_len > 0)
    for (int p = l; p < M / list_len; p += 64) bnd = fminf(bnd, lv[p * list_len + list_len - 1]);

  float ev[MAXP];
  int ei[MAXP];
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 64 + l;
    float v = INFINITY;
    int ix = INT_MAX;
    if (e < nval) {
      const int ii = lix[e];
      if (ii >= 0 && ii < nc) {
        v = lv[e];
        ix = ii;
      }
    }
    ev[p] = v;
    ei[p] = ix;
  }
  // Approximate top-LIST of the union, ordered by (approx, idx).
  float last = INFINITY;
  if (rank_merge) {
    // Rank merge: every entry's rank = the number of entries lexicographically below it,
    // counted against all M entries read back from LDS (broadcast reads, no dependent chain);
    // entries of rank < LIST land in sel[rank].  Same selection as the argmin rounds below.
#pragma unroll
    for (int p = 0; p < kRM; ++p)
      sent[w][p * 64 + l] = make_float2(ev[p], __int_as_float(ei[p]));
    if (l < LIST) sel[w][l] = -1;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    int rk[MAXP];
#pragma unroll
    for (int p = 0; p < MAXP; ++p) rk[p] = 0;
    const int mtot = min(nval, 64 * kRM);
#pragma nounroll
    for (int e = 0; e < mtot; ++e) {
      const float2 o = sent[w][e];
      const float ov = o.x;
      const int oi = __float_as_int(o.y);
#pragma unroll
      for (int p = 0; p < MAXP; ++p) rk[p] += lex_less_f(ov, oi, ev[p], ei[p]) ? 1 : 0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < MAXP; ++p) {
      if (ei[p] != INT_MAX && rk[p] < LIST) {
        sel[w][rk[p]] = ei[p];
        selv[w][rk[p]] = ev[p];
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int s_last = sel[w][LIST - 1];
    last = (s_last >= 0) ? selv[w][LIST - 1] : INFINITY;
  }
#pragma nounroll
  for (int r = 0; r < (rank_merge ? 0 : LIST); ++r) {
    float bv = ev[0];
    int bi = ei[0];
#pragma unroll
    for (int p = 1; p < MAXP; ++p)
      if (lex_less_f(ev[p], ei[p], bv, bi)) {
        bv = ev[p];
        bi = ei[p];
      }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float ov = __shfl_xor(bv, m, kWave);
      const int oi = __shfl_xor(bi, m, kWave);
      if (lex_less_f(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
#pragma unroll
    for (int p = 0; p < MAXP; ++p)
      if (ei[p] == bi) ev[p] = INFINITY, ei[p] = INT_MAX;
    if (l == 0) sel[w][r] = (bi == INT_MAX) ? -1 : bi;
    last = bv;
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) bnd = fminf(bnd, __shfl_xor(bnd, m, kWave));
  bnd = fminf(bnd, last);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  // |q|^2 and the selection's error bound E (certification below; any summation order)
  const float* xq = query + q * d;
  double qn2 = 0.0;
  for (int f = l; f < d; f += 64) qn2 += (double)xq[f] * (double)xq[f];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) qn2 += __shfl_xor(qn2, m, kWave);
  const double cmax = (double)__uint_as_float(*cmax_bits);
  // e_terms * 2^-24 * (C^2 + 2 C |q|) bounds the selection's error (f32 path: 4 (d + 1);
  // split-f16 path: 2 (3 K + 16 + d), see make_plan), C = max candidate norm.
  const double E = (double)e_terms * 5.9604644775390625e-08 *
                       (cmax * cmax + 2.0 * cmax * sqrt(qn2)) + 1e-300;
  // Rank merge: only the candidates within the error band of the (k+1)-th approximate value
  // need exact distances.  Ranks >= mcut all have approx > v_(k+1) + 2.5 E: their exact d^2
  // exceeds every exact d^2 of the first k+1 (each within E of its approx), and the first
  // excluded value joins the certification bound, as the LIST-th did.
  int mcut = LIST;
  if (rank_merge && sel[w][kp1 - 1] >= 0) {
    const double cut = (double)selv[w][kp1 - 1] + 2.5 * E;
    const bool out = l >= kp1 && l < LIST && sel[w][l] >= 0 && (double)selv[w][l] > cut;
    const unsigned long long ob = __ballot(out);
    if (ob) {
      mcut = __builtin_ctzll(ob);  // ranks are sorted: the first excluded one
      bnd = fminf(bnd, selv[w][mcut]);
    }
  }

  // Exact f64 distances for the selected candidates, one per lane.
  double dd = INFINITY;
  int di = INT_MAX;
  if (l < mcut) {
    const int c = sel[w][l];
    if (c >= 0) {
      dd = exact_d2(xq, cand + (int64_t)c * d, d);
      di = c;
    }
  }
  // Bitonic sort of 64 (dd, di) pairs across the wave, ascending.
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride >= 1; stride >>= 1) {
      const double od = __shfl_xor(dd, stride, kWave);
      const int oi = __shfl_xor(di, stride, kWave);
      const bool up = ((l & size) == 0);
      const bool lower = ((l & stride) == 0);
      const bool other_less = lex_less(od, oi, dd, di);
      // lower lane keeps the min if ascending block, max otherwise
      const bool take = (lower == up) ? other_less : !other_less && !(od == dd && oi == di);
      if (take) {
        dd = od;
        di = oi;
      }
    }
  }
  // Certification: every candidate outside the exactly evaluated set has exact
  // d^2 >= bnd + |q|^2 - E.
  const double ek = __shfl(dd, kp1 - 1, kWave);
  const int eki = __shfl(di, kp1 - 1, kWave);
  bool ok = (eki != INT_MAX) && !overflow;
  if (bnd < 1e29f) ok = ok && (ek < ((double)bnd + qn2) - E);
  if (l < kp1) {
    Dout[q * kp1 + l] = sqrt_rn(dd);
    if (I64) I64[q * kp1 + l] = di;
    if (I32) I32[(int64_t)l * nq + q] = di;  // transposed [kp1][nq]
  }
  if (!ok && l == 0) {
    const int slot = atomicAdd(flag_count, 1);
    flag_list[slot] = (int)q;
  }
}

// ---------------------------------------------------------------------------------------
// 4. exhaustive exact fallback for uncertified queries
// ---------------------------------------------------------------------------------------
template <int LIST>
__global__ __launch_bounds__(256) void exact_kernel(const float* __restrict__ cand, int64_t nc,
                                                    const float* __restrict__ query, int64_t nq,
                                                    int d, int kp1,
                                                    const int* __restrict__ flag_count,
                                                    const int* __restrict__ flag_list,
                                                    double* __restrict__ Dout,
                                                    int64_t* __restrict__ I64,
                                                    int32_t* __restrict__ I32) {
  __shared__ double red_d[4];
  __shared__ int red_i[4];
  const int tid = threadIdx.x;
  const int l = tid & 63, w = tid >> 6;
  const int count = *flag_count;
  for (int fi = blockIdx.x; fi < count; fi += gridDim.x) {
    const int64_t q = flag_list[fi];
    const float* xq = query + q * d;
    double ld[LIST];
    int li[LIST];
#pragma unroll
    for (int j = 0; j < LIST; ++j) {
      ld[j] = INFINITY;
      li[j] = INT_MAX;
    }
#pragma nounroll
    for (int64_t c = tid; c < nc; c += blockDim.x) {
      const double x = exact_d2(xq, cand + c * d, d);
      const int xi = (int)c;
      if (lex_less(x, xi, ld[LIST - 1], li[LIST - 1])) {
        bool cc[LIST];
#pragma unroll
        for (int j = 0; j < LIST; ++j) cc[j] = lex_less(x, xi, ld[j], li[j]);
#pragma unroll
        for (int j = LIST - 1; j >= 1; --j) {
          ld[j] = cc[j - 1] ? ld[j - 1] : (cc[j] ? x : ld[j]);
          li[j] = cc[j - 1] ? li[j - 1] : (cc[j] ? xi : li[j]);
        }
        ld[0] = cc[0] ? x : ld[0];
        li[0] = cc[0] ? xi : li[0];
      }
    }
    // kp1 rounds of block argmin over list heads; the winner pops its head.
#pragma nounroll
    for (int r = 0; r < kp1; ++r) {
      double bd = ld[0];
      int bi = li[0];
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        const double od = __shfl_xor(bd, m, kWave);
        const int oi = __shfl_xor(bi, m, kWave);
        if (lex_less(od, oi, bd, bi)) {
          bd = od;
          bi = oi;
        }
      }
      if (l == 0) {
        red_d[w] = bd;
        red_i[w] = bi;
      }
      __syncthreads();
      bd = red_d[0];
      bi = red_i[0];
#pragma unroll
      for (int u = 1; u < 4; ++u)
        if (lex_less(red_d[u], red_i[u], bd, bi)) {
          bd = red_d[u];
          bi = red_i[u];
        }
      __syncthreads();
      if (li[0] == bi) {
#pragma unroll
        for (int j = 0; j < LIST - 1; ++j) {
          ld[j] = ld[j + 1];
          li[j] = li[j + 1];
        }
        ld[LIST - 1] = INFINITY;
        li[LIST - 1] = INT_MAX;
      }
      if (tid == 0) {
        Dout[q * kp1 + r] = sqrt_rn(bd);
        if (I64) I64[q * kp1 + r] = bi;
        if (I32) I32[(int64_t)r * nq + q] = bi;  // transposed [kp1][nq]
      }
    }
  }
}

__global__ void fill_identity_kernel(int* s, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) s[0] = (int)n;
  if (i < n) s[1 + i] = (int)i;
}

// ---------------------------------------------------------------------------------------
// host-side plan + dispatch
// ---------------------------------------------------------------------------------------
struct Plan {
  int d, kp1, KS, KSP, LIST, split, maxp;
  int mode;       // 0: f32 MFMA selection, 1: split-f16 MFMA selection (default, d + 1 <= 64)
  int KS16;       // k-steps of 16 (mode 1)
  int e_terms;    // selection error bound multiplier (refine certification)
  int sample;     // mode 1: tile stride of the sampling pass that seeds each query's bound (0: off)
  int filter;     // mode 1 + sampling: survivor filter pass (filter16_kernel) instead of lists
  int tau_list;   // list length of the sampling pass: >= ceil(kp1 / 2)
  int keep;       // split-f16 lists: per-half entries behind the union prune bound (0: off)
  int LIST16;     // split-f16 select: per-half list length (refine keeps LIST >= kp1 + 4)
  int M;          // refine input entries per query (lists: 2*split*LIST; filter: capacity)
  int list_len;   // refine: length of each ascending partial list (0: unsorted survivors)
  int64_t nc, nq, nct, nqt, tiles_per_split;
  size_t off_apack, off_scalars, off_lv, off_li, off_flag, off_tau, off_cnt, total;
};

static const int kKSChoices[] = {2, 4, 8, 12, 15, 16, 24, 32};
static const int kListChoices[] = {8, 16, 24, 32, 40, 64};

static int make_plan(int64_t nc, int64_t nq, int d, int kp1, int split_hint, Plan* P) {
  if (nc <= 0 || nq < 0 || d <= 0 || kp1 <= 0) {
    set_error("mepol_knn: bad sizes nc=%lld nq=%lld d=%d kp1=%d", (long long)nc, (long long)nq, d,
              kp1);
    return kErrBadArg;
  }
  if (kp1 > nc) {
    set_error("mepol_knn: n_neighbors=%d > n_samples=%lld (sklearn raises the same)", kp1,
              (long long)nc);
    return kErrBadArg;
  }
  if (nc > INT_MAX - 64) {
    set_error("mepol_knn: n_cand=%lld exceeds int32 indexing", (long long)nc);
    return kErrUnsupported;
  }
  const int need_ks = (d + 1 + 1) / 2;
  int KS = -1;
  for (int v : kKSChoices)
    if (v >= need_ks) {
      KS = v;
      break;
    }
  int LIST = -1;
  for (int v : kListChoices)
    if (v >= kp1 + 4 || (v == 64 && kp1 <= 60)) {
      LIST = v;
      break;
    }
  if (KS < 0 || LIST < 0) {
    set_error("mepol_knn: unsupported d=%d / k+1=%d (fast path supports d<=63, k+1<=60)", d, kp1);
    return kErrUnsupported;
  }
  P->d = d;
  P->kp1 = kp1;
  {
    const char* prec = getenv("MEPOL_KNN_PRECISION");
    const bool want_f32 = prec && (prec[0] == 'f' && prec[1] == '3' && prec[2] == '2');
    P->KS16 = (d + 1 + 15) / 16;
    // split-f16 lists: each half-lane keeps LIST16 entries and prunes against the union bound
    // (flush_buffer, keep = ceil(kp1/2) + 2 per half: 2 keep >= kp1 + 3).  A half holding more
    // than LIST16 of the query's nearest candidates only costs certification (exact path).
    P->keep = (kp1 + 1) / 2 + 2;
    P->LIST16 = 64;
    for (int v : kListChoices)
      if (v >= P->keep + 4) {
        P->LIST16 = v;
        break;
      }
    // split-f16 instantiations that stay below the 256-VGPR cap (at the cap the fragment
    // buffers of the asm-load pipeline are no longer safe from register copies)
    // (<3, 40> and every KS16 = 4 list size needed for kp1 > 21 reach the cap: excluded)
    // KS16 = 4 runs a double-buffered pipeline (select16_kernel, NB = 2) with lists <= 32
    const bool fits = (P->KS16 <= 3 && P->LIST16 <= (P->KS16 == 3 ? 32 : 40)) ||
                      (P->KS16 == 4 && P->LIST16 <= 32);
    P->mode = (!want_f32 && fits) ? 1 : 0;
    // f32: d + 1 fma-chain roundings, x4 margin.  split-f16: 3 K products per output summed in
    // f32 (<= 3K roundings), operand splitting 3 * 2^-22 = 12 * 2^-24, |c|^2 in f32 (d), x2.
    P->e_terms = P->mode ? 2 * (3 * 16 * P->KS16 + 16 + d) : 4 * (d + 1);
    // Sampling pass: every S-th candidate tile (MEPOL_KNN_SAMPLE=S, off by default: at C3 the
    // survivor filter measured slower than the list selection); only worth it when the sample
    // still holds many tiles.
    const char* smp = getenv("MEPOL_KNN_SAMPLE");
    int S = smp ? atoi(smp) : 0;
    const int64_t nct = (nc + 31) / 32;
    if (S < 2 || P->mode != 1 || P->KS16 > 3 || nct / S < 8 || (int64_t)32 * (nct / S) < 4 * kp1)
      S = 0;
    P->sample = S;
    P->tau_list = 64;
    for (int v : kListChoices)
      if (v >= (kp1 + 1) / 2) {
        P->tau_list = v;
        break;
      }
    const char* flt = getenv("MEPOL_KNN_FILTER");
    P->filter = (S > 0 && !(flt && flt[0] == '0')) ? 1 : 0;
  }
  P->KS = KS;
  P->KSP = (KS + 3) / 4 * 4;
  if (P->mode != 1 || P->filter) P->keep = 0;
  P->LIST = LIST;
  P->nc = nc;
  P->nq = nq;
  P->nct = (nc + 31) / 32;
  P->nqt = (nq + 31) / 32;
  int split = split_hint;
  if (split <= 0 && P->mode == 1 && P->filter) {
    // filter pass: 8 candidate ranges, one per XCD (filter16's block mapping), each small
    // enough for that XCD's L2 (25.6 MB of fragments at C3 -> 3.2 MB per XCD)
    split = 8;
    while (split > 1 && P->nct / split < 16) split >>= 1;
  } else if (split <= 0) {
    // enough waves to fill 256 CUs x 2 waves/SIMD several times over, tiles >= 16 per split.
    // Every (query, split) pays the list warm-up (the prune bound starts at +inf), so fewer,
    // longer ranges win once the chip is full: C3 split 2 = 12.9 ms, 3 = 13.4, 8 = 17.2
    // (tools/knn_splits.sh).  The split-f16 lists keep >= 2 ranges (one range of 24-entry half
    // lists certifies too few queries).
    const int64_t target = P->mode == 1 ? 12500 : 16384;
    split = (int)std::min<int64_t>(kMaxSplit, std::max<int64_t>(1, (target + P->nqt - 1) / std::max<int64_t>(P->nqt, 1)));
    if (P->mode == 1) split = std::max(split, 2);
    while (split > 1 && P->nct / split < 16) --split;
  }
  split = std::max(1, std::min(split, kMaxSplit));
  P->split = split;
  P->tiles_per_split = (P->nct + split - 1) / split;
  if (P->filter) {
    // survivors of the sampled bound: ~S*kp1 expected per query (S = 16 -> ~500 at k+1 = 31),
    // capacity 32*kp1 (>= 256); an overflowing query is answered by the exhaustive path
    const char* capv = getenv("MEPOL_KNN_CAP");
    const int cap = capv ? atoi(capv) : 32 * kp1;
    P->M = (int)align_up((size_t)std::max(256, std::min(cap, 2048)), 64);
    P->list_len = 0;
  } else {
    const int sel_list = P->mode == 1 ? P->LIST16 : LIST;
    P->M = 2 * split * sel_list;
    P->list_len = sel_list;
  }
  P->maxp = (P->M + 63) / 64;
  if (P->maxp > 32) {
    set_error("mepol_knn: refine capacity %d entries per query exceeds 2048", P->M);
    return kErrUnsupported;
  }
  size_t off = 0;
  P->off_apack = off;
  off = align_up(off + std::max((size_t)P->nct * 64 * P->KSP * sizeof(float),
                                (size_t)P->nct * 64 * P->KS16 * 16 * sizeof(_Float16)),
                 256);
  P->off_scalars = off;  // [0] max |c| bits, [1] fallback count, [2] max |q| bits, [4..5] invalid rows
  off = align_up(off + 32, 256);
  const size_t nl = (size_t)std::max<int64_t>(nq, 1) * P->M;
  P->off_lv = off;
  off = align_up(off + nl * sizeof(float), 256);
  P->off_li = off;
  off = align_up(off + nl * sizeof(int), 256);
  P->off_flag = off;
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(int), 256);
  P->off_tau = off;
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(float), 256);
  P->off_cnt = off;
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(int), 256);
  P->total = off;
  return 0;
}

template <int KS>
static void launch_select_ks(const Plan& P, dim3 g, const float* ap, const float* query, float* lv,
                             int* li, hipStream_t st) {
  constexpr int KSP = (KS + 3) / 4 * 4;
  switch (P.LIST) {
    case 8:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 8>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
    case 16:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 16>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
    case 24:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 24>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
    case 32:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 32>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
    case 40:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 40>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
    default:
      hipLaunchKernelGGL((select_kernel<KS, KSP, 64>), g, dim3(256), 0, st, ap, query, P.nq, P.d,
                         P.nct, P.split, P.tiles_per_split, lv, li);
      break;
  }
}

// tau_pass: the sampling pass (split 1, every P.sample-th tile) writing tau; otherwise the main
// selection, seeded by tau when it is non-null.
template <int KS16>
static void launch_select16_ks(const Plan& P, const _Float16* ap, const float* query,
                               const unsigned* scal, float* tau, bool tau_pass, float* lv, int* li,
                               hipStream_t st) {
  const unsigned gx = (unsigned)((P.nqt + 3) / 4);
  if (tau_pass) {
    const int64_t ns = (P.nct + P.sample - 1) / P.sample;
#define MEPOL_TAU16(L)                                                                           \
  hipLaunchKernelGGL((select16_kernel<KS16, L, true>), dim3(gx, 1), dim3(256), 0, st, ap, query, \
                     P.nq, P.d, ns, 1, ns, P.sample, P.kp1, 0, scal, nullptr, tau, nullptr, nullptr)
    switch (P.tau_list) {  // >= ceil(kp1 / 2), kp1 <= 60
      case 8: MEPOL_TAU16(8); break;
      case 16: MEPOL_TAU16(16); break;
      case 24: MEPOL_TAU16(24); break;
      default: MEPOL_TAU16(32); break;
    }
#undef MEPOL_TAU16
    return;
  }
#define MEPOL_SEL16(L)                                                                            \
  hipLaunchKernelGGL((select16_kernel<KS16, L, false>), dim3(gx, (unsigned)P.split), dim3(256), 0, \
                     st, ap, query, P.nq, P.d, P.nct, P.split, P.tiles_per_split, 1, P.kp1, P.keep, \
                     scal, tau, nullptr, lv, li)
  switch (P.LIST16) {  // >= keep + 4 >= 7; mode 1 needs LIST16 <= 40
    case 8: MEPOL_SEL16(8); break;
    case 16: MEPOL_SEL16(16); break;
    case 24: MEPOL_SEL16(24); break;
    case 32: MEPOL_SEL16(32); break;
    default: MEPOL_SEL16(40); break;
  }
#undef MEPOL_SEL16
}

// MEPOL_KNN_RANK_MERGE=0 selects the argmin-round merge in refine_kernel (A/B probe).
static int refine_rank_merge() {
  static const int v = [] {
    const char* e = getenv("MEPOL_KNN_RANK_MERGE");
    return e ? atoi(e) : 1;
  }();
  return v;
}

// KS16 = 4 (d + 1 in 49..64): double-buffered select16 with lists of at most 32, no sampling
// pass (make_plan)
static void launch_select16_ks4(const Plan& P, const _Float16* ap, const float* query,
                                const unsigned* scal, float* tau, float* lv, int* li,
                                hipStream_t st) {
  const unsigned gx = (unsigned)((P.nqt + 3) / 4);
#define MEPOL_SEL16W(L)                                                                          \
  hipLaunchKernelGGL((select16_kernel<4, L, false>), dim3(gx, (unsigned)P.split), dim3(256), 0, \
                     st, ap, query, P.nq, P.d, P.nct, P.split, P.tiles_per_split, 1, P.kp1, P.keep, \
                     scal, tau, nullptr, lv, li)
  switch (P.LIST16) {
    case 8: MEPOL_SEL16W(8); break;
    case 16: MEPOL_SEL16W(16); break;
    case 24: MEPOL_SEL16W(24); break;
    default: MEPOL_SEL16W(32); break;
  }
#undef MEPOL_SEL16W
}

template <int LIST>
static void launch_refine_list(const Plan& P, const float* cand, const float* query,
                               const float* lv, const int* li, const unsigned* cmax,
                               const float* tau, const int* counts, double* D, int64_t* I64,
                               int32_t* I32, int* fc, int* fl, hipStream_t st) {
  dim3 g((unsigned)((P.nq + 3) / 4));
  // MAXP = ceil(M / 64) <= 32
  if (P.maxp <= 2)
    hipLaunchKernelGGL((refine_kernel<LIST, 2>), g, dim3(256), 0, st, cand, P.nc, query, P.nq, P.d,
                       P.kp1, P.M, P.list_len, counts, lv, li, cmax, P.e_terms, tau, D, I64, I32, fc, fl, refine_rank_merge());
  else if (P.maxp <= 4)
    hipLaunchKernelGGL((refine_kernel<LIST, 4>), g, dim3(256), 0, st, cand, P.nc, query, P.nq, P.d,
                       P.kp1, P.M, P.list_len, counts, lv, li, cmax, P.e_terms, tau, D, I64, I32, fc, fl, refine_rank_merge());
  else if (P.maxp <= 8)
    hipLaunchKernelGGL((refine_kernel<LIST, 8>), g, dim3(256), 0, st, cand, P.nc, query, P.nq, P.d,
                       P.kp1, P.M, P.list_len, counts, lv, li, cmax, P.e_terms, tau, D, I64, I32, fc, fl, refine_rank_merge());
  else if (P.maxp <= 16)
    hipLaunchKernelGGL((refine_kernel<LIST, 16>), g, dim3(256), 0, st, cand, P.nc, query, P.nq,
                       P.d, P.kp1, P.M, P.list_len, counts, lv, li, cmax, P.e_terms, tau, D, I64, I32, fc, fl, refine_rank_merge());
  else
    hipLaunchKernelGGL((refine_kernel<LIST, 32>), g, dim3(256), 0, st, cand, P.nc, query, P.nq,
                       P.d, P.kp1, P.M, P.list_len, counts, lv, li, cmax, P.e_terms, tau, D, I64, I32, fc, fl, refine_rank_merge());
}

template <int LIST>
static void launch_exact_list(const Plan& P, const float* cand, const float* query, const int* fc,
                              const int* fl, double* D, int64_t* I64, int32_t* I32,
                              unsigned grid, hipStream_t st) {
  hipLaunchKernelGGL((exact_kernel<LIST>), dim3(grid), dim3(256), 0, st, cand, P.nc, query, P.nq,
                     P.d, P.kp1, fc, fl, D, I64, I32);
}

}  // namespace knn
}  // namespace mepol

using namespace mepol;
using namespace mepol::knn;

extern "C" int mepol_knn_workspace_size(int64_t n_cand, int64_t n_query, int d, int kp1,
                                        int split_hint, size_t* bytes) {
  Plan P;
  int rc = make_plan(n_cand, n_query, d, kp1, split_hint, &P);
  if (rc) return rc;
  *bytes = P.total;
  return 0;
}

extern "C" int mepol_knn_plan_info(int64_t n_cand, int64_t n_query, int d, int kp1,
                                   int split_hint, int* ks, int* list, int* split) {
  Plan P;
  int rc = make_plan(n_cand, n_query, d, kp1, split_hint, &P);
  if (rc) return rc;
  if (ks) *ks = P.KS;
  if (list) *list = P.LIST;
  if (split) *split = P.split;
  return 0;
}

extern "C" int mepol_knn(const float* cand, int64_t n_cand, const float* query, int64_t n_query,
                         int d, int kp1, int split_hint, double* dist_out, int64_t* idx_out,
                         int32_t* idx32_out, int32_t* n_fallback_out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  Plan P;
  int rc = make_plan(n_cand, n_query, d, kp1, split_hint, &P);
  if (rc) return rc;
  if (!cand || !query || !dist_out || !workspace) {
    set_error("mepol_knn: null pointer argument");
    return kErrBadArg;
  }
  if (workspace_bytes < P.total) {
    set_error("mepol_knn: workspace %zu bytes < required %zu", workspace_bytes, P.total);
    return kErrWorkspace;
  }
  if (n_query == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  float* apack = (float*)(ws + P.off_apack);
  unsigned* cmax = (unsigned*)(ws + P.off_scalars);
  int* fcount = n_fallback_out ? (int*)n_fallback_out : (int*)(ws + P.off_scalars + 4);
  float* lv = (float*)(ws + P.off_lv);
  int* li = (int*)(ws + P.off_li);
  int* flist = (int*)(ws + P.off_flag);

  float* tau = nullptr;   // sampled per-query bounds (mode 1 with sampling)
  int* counts = nullptr;  // survivors per query (filter pass)
  MEPOL_HIP(hipMemsetAsync(ws + P.off_scalars, 0, 32, st));
  if (n_fallback_out) MEPOL_HIP(hipMemsetAsync(n_fallback_out, 0, sizeof(int32_t), st));
  // scal[0] = max candidate norm (refine's C), scal[2] = max query norm (split-f16 scale)
  hipLaunchKernelGGL(norms_kernel, dim3((unsigned)((P.nc + 255) / 256)), dim3(256), 0, st, cand,
                     P.nc, P.d, cmax, cmax + 4);
  hipLaunchKernelGGL(norms_kernel, dim3((unsigned)((P.nq + 255) / 256)), dim3(256), 0, st, query,
                     P.nq, P.d, cmax + 2, cmax + 4);
  MEPOL_CHECK_LAUNCH();
  {
    // sklearn rejects non-finite input (ValueError from check_array): validate before the scan.
    // One stream synchronisation per call, like the reference's blocking kneighbors.
    unsigned bad[2] = {0, 0};
    MEPOL_HIP(hipMemcpyAsync(bad, cmax + 4, sizeof(bad), hipMemcpyDeviceToHost, st));
    MEPOL_HIP(hipStreamSynchronize(st));
    if (bad[0]) {
      set_error("mepol_knn: Input contains NaN or infinity (%u rows)", bad[0]);
      return kErrBadArg;
    }
    if (bad[1]) {
      set_error("mepol_knn: %u rows have a squared norm beyond float32 range", bad[1]);
      return kErrUnsupported;
    }
  }
  if (P.mode == 1) {
    _Float16* ap16 = (_Float16*)apack;
    const int64_t total = P.nct * 64;
    hipLaunchKernelGGL(pack16_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                       cand, P.nc, P.d, P.KS16, P.nct, ap16, cmax);
    MEPOL_CHECK_LAUNCH();
    tau = P.sample ? (float*)(ws + P.off_tau) : nullptr;
    if (P.filter) {
      counts = (int*)(ws + P.off_cnt);
      MEPOL_HIP(hipMemsetAsync(counts, 0, (size_t)P.nq * sizeof(int), st));
    }
    for (int pass = tau ? 0 : 1; pass < 2; ++pass) {
      if (pass == 1 && P.filter) {
        const dim3 g((unsigned)((P.nqt + 3) / 4), (unsigned)P.split);
#define MEPOL_FLT16(K)                                                                          \
  hipLaunchKernelGGL((filter16_kernel<K>), g, dim3(256), 0, st, ap16, query, P.nq, P.d, P.nct,  \
                     P.split, P.tiles_per_split, cmax, tau, P.M, counts, lv, li)
        switch (P.KS16) {
          case 1: MEPOL_FLT16(1); break;
          case 2: MEPOL_FLT16(2); break;
          default: MEPOL_FLT16(3); break;
        }
#undef MEPOL_FLT16
        MEPOL_CHECK_LAUNCH();
        continue;
      }
      switch (P.KS16) {  // mode 1 only for KS16 <= 3, or 4 with lists <= 32 (make_plan)
        case 1: launch_select16_ks<1>(P, ap16, query, cmax, tau, pass == 0, lv, li, st); break;
        case 2: launch_select16_ks<2>(P, ap16, query, cmax, tau, pass == 0, lv, li, st); break;
        case 3: launch_select16_ks<3>(P, ap16, query, cmax, tau, pass == 0, lv, li, st); break;
        default: launch_select16_ks4(P, ap16, query, cmax, tau, lv, li, st); break;
      }
      MEPOL_CHECK_LAUNCH();
    }
  } else {
    const int64_t total = P.nct * 64;
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, cand,
                       P.nc, P.d, P.KSP, P.nct, apack, cmax);
    MEPOL_CHECK_LAUNCH();
    dim3 g((unsigned)((P.nqt + 3) / 4), (unsigned)P.split);
    switch (P.KS) {
      case 2: launch_select_ks<2>(P, g, apack, query, lv, li, st); break;
      case 4: launch_select_ks<4>(P, g, apack, query, lv, li, st); break;
      case 8: launch_select_ks<8>(P, g, apack, query, lv, li, st); break;
      case 12: launch_select_ks<12>(P, g, apack, query, lv, li, st); break;
      case 15: launch_select_ks<15>(P, g, apack, query, lv, li, st); break;
      case 16: launch_select_ks<16>(P, g, apack, query, lv, li, st); break;
      case 24: launch_select_ks<24>(P, g, apack, query, lv, li, st); break;
      default: launch_select_ks<32>(P, g, apack, query, lv, li, st); break;
    }
    MEPOL_CHECK_LAUNCH();
  }
  switch (P.LIST) {
    case 8: launch_refine_list<8>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
    case 16: launch_refine_list<16>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
    case 24: launch_refine_list<24>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
    case 32: launch_refine_list<32>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
    case 40: launch_refine_list<40>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
    default: launch_refine_list<64>(P, cand, query, lv, li, cmax, tau, counts, dist_out, idx_out, idx32_out, fcount, flist, st); break;
  }
  MEPOL_CHECK_LAUNCH();
  const unsigned eg = 512;
  switch (P.LIST) {
    case 8: launch_exact_list<8>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
    case 16: launch_exact_list<16>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
    case 24: launch_exact_list<24>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
    case 32: launch_exact_list<32>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
    case 40: launch_exact_list<40>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
    default: launch_exact_list<64>(P, cand, query, fcount, flist, dist_out, idx_out, idx32_out, eg, st); break;
  }
  MEPOL_CHECK_LAUNCH();
  return 0;
}

// Exhaustive exact k-NN for every query (no fp32 selection): the reference semantics at the
// cost of a full f64 scan.  Used for d > 63 / k+1 > 60 and as an independent check.
extern "C" int mepol_knn_exact(const float* cand, int64_t n_cand, const float* query,
                               int64_t n_query, int d, int kp1, double* dist_out, int64_t* idx_out,
                               int32_t* idx32_out, int32_t* scratch_idx, void* stream) {
  if (n_cand <= 0 || n_query < 0 || d <= 0 || kp1 <= 0 || kp1 > 64 || kp1 > n_cand ||
      !scratch_idx) {
    set_error("mepol_knn_exact: bad arguments (needs k+1 <= 64, k+1 <= n_cand, scratch)");
    return kErrBadArg;
  }
  if (n_query == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // scratch_idx: [1 + n_query] int32: count, then the identity query list.
  Plan P{};
  P.nc = n_cand;
  P.nq = n_query;
  P.d = d;
  P.kp1 = kp1;
  hipLaunchKernelGGL(fill_identity_kernel, dim3((unsigned)((n_query + 255) / 256)), dim3(256), 0, st, scratch_idx,
                     n_query);
  MEPOL_CHECK_LAUNCH();
  const unsigned grid = (unsigned)std::min<int64_t>(n_query, 4096);
  if (kp1 <= 8)
    launch_exact_list<8>(P, cand, query, scratch_idx, scratch_idx + 1, dist_out, idx_out, idx32_out, grid, st);
  else if (kp1 <= 16)
    launch_exact_list<16>(P, cand, query, scratch_idx, scratch_idx + 1, dist_out, idx_out, idx32_out, grid, st);
  else if (kp1 <= 40)
    launch_exact_list<40>(P, cand, query, scratch_idx, scratch_idx + 1, dist_out, idx_out, idx32_out, grid, st);
  else
    launch_exact_list<64>(P, cand, query, scratch_idx, scratch_idx + 1, dist_out, idx_out, idx32_out, grid, st);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
