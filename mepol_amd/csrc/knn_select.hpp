// The k-NN selection kernel (step 2 of knn.hip's pipeline), built once per k-step count by
// knn_select_ks{1..4}.hip.
#pragma once
#include "knn_common.hpp"

namespace mepol {
namespace knn {

// Per-query state of a lane: its sorted top-LIST list (values ascending), the prune bound, the
// seed it started from and the fill of its LDS group buffer.
template <int LIST>
struct LaneList {
  float ld[LIST];
  int li[LIST];
  float thr, thr0;
  int cnt;
};

// Row-group entries per lane in the LDS group buffer: 10 (51.2 KB per workgroup, still 3 per
// CU); a fuller buffer makes fuller flushes: C3 select 4.96 -> 4.78 ms against 8, 5.43 at 6
// (profiles/r5/knn/grpcap_ab.txt)
constexpr int kGrpCap = 10;

// The lane's group buffer into its sorted list.  A hit row group is buffered whole (its four
// values and the candidate index of its first row), so recording it costs the wave one address
// and one cursor step; here each entry gives up its values under the lane's bound smallest
// first, one insertion pass per value that some lane of the wave still has (usually one per
// entry).  Then the prune bound is shared with the partner lane (l ^ 32 serves the same query
// column): the tighter of their list maxima, and with keep > 0 also max(own keep-th,
// partner's keep-th) -- the two half lists then hold >= 2 keep values at or below it, so
// 2 keep >= kp1 + 3 of the query's candidates in this range are never pruned.  The bound only
// decreases over the scan.  Every lane of the wave calls it.
template <int LIST>
__device__ __forceinline__ void flush_groups(float (&ld)[LIST], int (&li)[LIST], float& thr,
                                             int& cnt, const f32x4 (*gv)[64],
                                             const int (*gt)[64], int l, float thr0, int keep) {
  const int mc = wave_max_i(cnt);
#pragma nounroll
  for (int e = 0; e < mc; ++e) {
    const f32x4 ev = gv[e][l];
    const int tag = gt[e][l];
    const bool own = e < cnt;
    float v0 = own ? ev[0] : INFINITY, v1 = own ? ev[1] : INFINITY;
    float v2 = own ? ev[2] : INFINITY, v3 = own ? ev[3] : INFINITY;
#pragma nounroll
    for (int pass = 0; pass < 4; ++pass) {
      const float x = fminf(fminf(v0, v1), fminf(v2, v3));
      if (!__ballot(x < thr)) break;  // wave-uniform
      const int i = v0 == x ? 0 : (v1 == x ? 1 : (v2 == x ? 2 : 3));  // its row: tag + i
      if (x < thr) {
        list_insert<LIST>(ld, li, x, tag + i);
        thr = ld[LIST - 1];
      }
      v0 = i == 0 ? INFINITY : v0;
      v1 = i == 1 ? INFINITY : v1;
      v2 = i == 2 ? INFINITY : v2;
      v3 = i == 3 ? INFINITY : v3;
    }
  }
  cnt = 0;
  thr = fminf(thr0, fminf(ld[LIST - 1], __shfl_xor(ld[LIST - 1], 32, kWave)));
  if (keep > 0) {
    const float kv = list_at<LIST>(ld, keep - 1);
    thr = fminf(thr, fmaxf(kv, __shfl_xor(kv, 32, kWave)));
  }
}

// B operands (queries) of lane l's query column: B[k = 16 s + 8h + j][col = l&31] = sigma q_f
// (f < d), 1 (f == d), 0, split into f16 hi + lo.  Unconditional loads at clamped addresses (a
// load under a per-element condition makes hipcc wait for each one in turn).
template <int KS16>
__device__ __forceinline__ void query_frags(const float* __restrict__ query, int64_t q, int64_t nq,
                                            int d, float sg, int h, f16x8 (&bhi)[KS16],
                                            f16x8 (&blo)[KS16]) {
  const bool qvalid = q < nq;
  const float* qrow = query + min(q, nq - 1) * d;
#pragma unroll
  for (int s = 0; s < KS16; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * s + 8 * h + j;
      const float x = qrow[min(f, d - 1)];  // finite (validated): x * 0 = 0
      const float v = ((f < d ? sg : 0.f) * x + (f == d ? 1.f : 0.f)) * (qvalid ? 1.f : 0.f);
      _Float16 a, b;
      split_f16(v, a, b);
      bhi[s][j] = a;
      blo[s][j] = b;
    }
}

// Partial top-LIST lists of every query over its split's tile range.  The queries are split into
// f16 hi + lo (2^-22 relative).  NH = 1 (candidate-hi, the default): the candidates are the f16
// hi halves of A and 2 MFMAs per k-step (A_hi q_hi + A_hi q_lo) accumulate in f32; the value's
// error is dominated by the candidate rounding, 2^-11 (|c|^2 + 2 |c||q|), and only the hi half
// travels (1 KB per k-step and tile).  With <= 3 k-steps the q_lo MFMA is dropped as well (one
// MFMA per k-step; the query rounding, 2^-11 2 |c||q|, joins the bound: make_plan).  NH = 2
// (split candidates): A_hi and A_lo travel and 3 MFMAs per k-step (+ A_lo q_hi) give
// ~f32-class values, 2 (3 K + 16 + d) 2^-24 (|c|^2 + 2 |c||q|),
// for data whose neighbour spacing is below the f16 band (make_plan).  refine's certification
// uses the plan's bound either way.
//
// One query tile of 32 per wave (one lane = one query column, 16 of each candidate tile's 32
// rows), four waves per workgroup.  The candidate fragments stream from L2 into every wave
// (1 KB per k-step, half and tile): at C3 the texture data path is the bound (TD busy ~ the
// kernel's CU-cycles, profiles/r5/knn/select_counters_C3_*.txt).  Tried and dropped in round 5
// (profiles/r5/knn/): two query tiles per wave (the lists then cap occupancy at 2 waves per
// SIMD), and the fragments shared through an LDS ring (3x less texture traffic, but a barrier
// per ring interval made the waves wait out each other's insertions; tools/variants/).
// OCC: waves per SIMD the VGPR budget is cut for (__launch_bounds__).
template <int KS16, int LIST, int NH, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void select16_kernel(
    const _Float16* __restrict__ apack, const float* __restrict__ query, int64_t nq, int d,
    int64_t nct, int split, int64_t tiles_per_split, int keep, const unsigned* __restrict__ scal,
    float* __restrict__ out_v, int* __restrict__ out_i, int* __restrict__ seed) {
  // group buffers: per lane kGrpCap x (4 values, first-row index)
  __shared__ f32x4 gbv[4][kGrpCap][64];
  __shared__ int gbt[4][kGrpCap][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: SGPR
  const int l = threadIdx.x & 63;
  // XCD-aware block mapping: workgroups go round-robin over the 8 XCDs by linear id, so with
  // sp = id % split (split a multiple of 8) every XCD only ever reads the candidate ranges
  // sp = xcd (mod 8), which then stay resident in that XCD's 4 MB L2.  Any other split (2 at
  // C3) keeps the split-major order: the blocks in flight then all read one candidate range.
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const bool xcd_map = (split & 7) == 0;
  const int sp = xcd_map ? (int)(lin % split) : (int)blockIdx.y;
  const int64_t qt0 = (xcd_map ? lin / split : (int64_t)blockIdx.x) * 4 + w;
  if (qt0 * 32 >= nq || (scal[4] | scal[5])) return;  // wave-uniform (rejected input: knn.hip)
  const int h = l >> 5;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);  // exact: sigma is a power of two
  constexpr bool kQueryLo = NH == 2 || KS16 >= 4;  // make_plan's bound covers the rest

  f16x8 bhi[KS16], blo[KS16];
  const int64_t q = qt0 * 32 + (l & 31);
  const bool qvalid = q < nq;
  query_frags<KS16>(query, q, nq, d, sg, h, bhi, blo);

  LaneList<LIST> S;
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    S.ld[j] = INFINITY;
    S.li[j] = -1;
  }
  // Seed of the prune bound: the tightest bound a range of this query already finished with
  // (the grid runs split-major, so range 0's blocks are mostly done when range 1's start).
  // Any value is sound -- a lane only claims what its own scan rejected against its own bound,
  // and refine certifies against the reported bounds -- and every published bound has
  // >= 2 keep candidates of its range at or below it, so it costs no certification.  It skips
  // most of the list warm-up, where the bulk of the insertions happen.  The lists (and so how
  // many queries refine certifies) depend on which ranges finished first; the certified
  // output does not.  System scope: the load and the publishing atomic below go past the
  // XCD's own L2.
  S.thr0 = INFINITY;
  if (seed && qvalid)
    S.thr0 = order_key_float(
        __hip_atomic_load(seed + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  S.thr = S.thr0;
  S.cnt = 0;

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  // Fragment ring in registers: tile t's MFMAs run while the next tiles' loads are in flight; a
  // buffer is refilled only after the chain that read it was issued.  Plain loads: hipcc
  // counts the waits (each step waits for the oldest tile in flight only).  A deeper ring
  // (4, 5) and a shallower one (2) measured the same or slower (profiles/r5/knn/).
  constexpr int NV = NH * KS16;  // dwordx4 per lane per tile: one per (k-step, half)
  constexpr int NB = 3;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + l;
  f32x4 Bf[NB][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) A[v] = p[v * 64];
  };
  auto chain = [&](const f32x4 (&A)[NV]) -> f32x16 {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KS16; ++s) {
      const f16x8 ah = __builtin_bit_cast(f16x8, A[NH * s]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhi[s], acc, 0, 0, 0);
      if constexpr (kQueryLo)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blo[s], acc, 0, 0, 0);
      if constexpr (NH == 2) {
        const f16x8 al = __builtin_bit_cast(f16x8, A[2 * s + 1]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhi[s], acc, 0, 0, 0);
      }
    }
    return acc;
  };
  auto process = [&](const f32x16& acc, int64_t t) {
    // min over the 4 row groups (rows 4g..4g+3 of the accumulator), then over the groups
    float gm[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      gm[g] = fminf(fminf(acc[4 * g], acc[4 * g + 1]), fminf(acc[4 * g + 2], acc[4 * g + 3]));
    const float m = fminf(fminf(gm[0], gm[1]), fminf(gm[2], gm[3]));
    if (__ballot(m < S.thr)) {
      // accumulator row 4g + i is candidate row tb + 8g + i of the tile (32x32 C/D map)
      const int tb = (int)(t * 32) + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (gm[g] < S.thr) {
          gbv[w][S.cnt][l] = f32x4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
          gbt[w][S.cnt][l] = tb + 8 * g;
          S.cnt += 1;
        }
      }
      // a tile adds <= 4 entries: the cursor enters every tile at <= kGrpCap - 4 (a check per
      // pair of row groups at kGrpCap - 2 measured slower: profiles/r5/knn/grpcap_ab.txt)
      if (__ballot(S.cnt > kGrpCap - 4))
        flush_groups<LIST>(S.ld, S.li, S.thr, S.cnt, gbv[w], gbt[w], l, S.thr0, keep);
    }
  };
  // Every chain's MFMA latency hides under the threshold work of the previous tile.
  f32x16 accP;
  auto step = [&](const f32x4 (&A)[NV], int64_t t, bool prev) {
    const f32x16 acc = chain(A);
    if (prev) process(accP, t - 1);
    accP = acc;
  };
  if (t0 < t1) {
    const int64_t tl = t1 - 1;
#pragma unroll
    for (int b = 0; b < NB - 1; ++b) load(Bf[b], min(t0 + b, tl));
    int64_t t = t0;
    // steady state, unrolled by NB so buffer indices are compile-time: tile t is in
    // Bf[(t - t0) % NB]; the buffer of tile t - 1 (its chain issued) takes tile t + NB - 1 (the
    // refills of the last tiles re-read tile t1 - 1).
    auto step_at = [&](int cur, bool prev) {
      load(Bf[(cur + NB - 1) % NB], min(t + NB - 1, tl));
      step(Bf[cur], t, prev);
      ++t;
    };
    step_at(0, false);
#pragma nounroll
    while (t + NB - 1 < t1) {
#pragma unroll
      for (int b = 1; b <= NB; ++b) step_at(b % NB, true);
    }
#pragma unroll
    for (int b = 1; b < NB; ++b)  // remainder (0..NB-1 tiles), same buffer rotation
      if (t < t1) step_at(b % NB, true);
    process(accP, t - 1);
  }

  flush_groups<LIST>(S.ld, S.li, S.thr, S.cnt, gbv[w], gbt[w], l, S.thr0, keep);
  // publish this range's final bound (the same in both lanes of the query)
  if (seed && qvalid && h == 0)
    __hip_atomic_fetch_min(seed + q, float_order_key(S.thr), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  if (qvalid) {
    // The last slot carries this lane's final bound: every candidate of its range that is not
    // in the list has an approximate value >= min(list last, thr) (rejected against thr, or
    // evicted from the list); a last entry at or above the bound is dropped (idx -1), the
    // bound covers it.  refine takes the min over the query's lanes.
    const float bound = fminf(S.ld[LIST - 1], S.thr);
    const int64_t o = ((q * split + sp) * 2 + h) * LIST;
#pragma unroll
    for (int j = 0; j < LIST - 1; ++j) {
      out_v[o + j] = S.ld[j] * inv_s2;
      out_i[o + j] = S.li[j];
    }
    out_v[o + LIST - 1] = bound * inv_s2;
    out_i[o + LIST - 1] = (bound < S.ld[LIST - 1]) ? -1 : S.li[LIST - 1];
  }
}


// ---------------------------------------------------------------------------------------
// Probe seeds (round 6).  Before the selection, every query's prune bound is seeded from a
// strided sample of kProbeTiles candidate tiles spread over the whole candidate set: per lane
// the kProbeKth-th smallest of its per-tile minima (each minimum is a distinct candidate's
// approximate value, so at least kProbeKth candidates lie at or below it), the smaller of the
// two lanes of the query goes to seed[q].  Without it the first candidate range of every query
// starts from +inf and pays the whole list warm-up, ~LIST ln(n / LIST) insertions per lane,
// the bulk of the select's list work; from the probe seed a range inserts only the candidates
// below the sample's quantile.  Any seed is sound (select16_kernel's seed comment); this one
// leaves ~8 / (32 kProbeTiles) of all candidates below it, far more than k + 1, so the lists
// still certify.
// ---------------------------------------------------------------------------------------

template <int KS16, int NH>
__global__ __launch_bounds__(256) void probe16_kernel(const _Float16* __restrict__ apack,
                                                      const float* __restrict__ query, int64_t nq,
                                                      int d, int64_t nct,
                                                      const unsigned* __restrict__ scal,
                                                      int* __restrict__ seed) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  const int64_t qt0 = (int64_t)blockIdx.x * 4 + w;
  if (qt0 * 32 >= nq || (scal[4] | scal[5])) return;  // wave-uniform
  const int h = l >> 5;
  const float sg = knn_scale(scal);
  constexpr bool kQueryLo = NH == 2 || KS16 >= 4;
  f16x8 bhi[KS16], blo[KS16];
  const int64_t q = qt0 * 32 + (l & 31);
  query_frags<KS16>(query, q, nq, d, sg, h, bhi, blo);
  constexpr int NV = NH * KS16;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + l;
  const int64_t np = min<int64_t>(kProbeTiles, nct);
  const int64_t stride = nct / np;  // >= 1
  float kth[kProbeKth];
#pragma unroll
  for (int j = 0; j < kProbeKth; ++j) kth[j] = INFINITY;
  constexpr int U = 4;  // tiles in flight
#pragma nounroll
  for (int64_t i0 = 0; i0 < np; i0 += U) {
    f32x4 A[U][NV];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t t = min(i0 + u, np - 1) * stride + stride / 2;
#pragma unroll
      for (int v = 0; v < NV; ++v) A[u][v] = abase[(t * NV + v) * 64];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x16 acc = {};
#pragma unroll
      for (int s = 0; s < KS16; ++s) {
        const f16x8 ah = __builtin_bit_cast(f16x8, A[u][NH * s]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhi[s], acc, 0, 0, 0);
        if constexpr (kQueryLo)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blo[s], acc, 0, 0, 0);
        if constexpr (NH == 2) {
          const f16x8 al = __builtin_bit_cast(f16x8, A[u][2 * s + 1]);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhi[s], acc, 0, 0, 0);
        }
      }
      float m = acc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) m = fminf(m, acc[r]);
      // the tile repeated by a clamped index (np % U) must not count twice
      if (i0 + u >= np) m = INFINITY;
      // branch-free insert into the ascending kth list
#pragma unroll
      for (int j = kProbeKth - 1; j >= 1; --j)
        kth[j] = m < kth[j - 1] ? kth[j - 1] : fminf(kth[j], m);
      kth[0] = fminf(kth[0], m);
    }
  }
  const float v = fminf(kth[kProbeKth - 1], __shfl_xor(kth[kProbeKth - 1], 32, kWave));
  if (q < nq && h == 0) seed[q] = float_order_key(v);
}

template <int KS16, int NH>
static void launch_probe16(const SelectArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((probe16_kernel<KS16, NH>), dim3((unsigned)((a.nqt + 3) / 4)), dim3(256), 0,
                     st, a.apack, a.query, a.nq, a.d, a.nct, a.scal, a.seed);
}


// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
template <int KS16, int NH>
static void launch_select16_ks(const SelectArgs& a, hipStream_t st) {
  const dim3 g((unsigned)((a.nqt + 3) / 4), (unsigned)a.split);
#define MEPOL_SEL16(L, O)                                                                       \
  hipLaunchKernelGGL((select16_kernel<KS16, L, NH, O>), g, dim3(256), 0, st, a.apack, a.query,  \
                     a.nq, a.d, a.nct, a.split, a.tiles_per_split, a.keep, a.scal, a.out_v,      \
                     a.out_i, a.seed)
  // 3 waves per SIMD also for 3-4 k-steps, despite a few spilled dwords there: 2 waves per
  // SIMD measured slower at d = 47 (6.14 -> 6.57 ms select; profiles/r5/knn/occ_ks3_ab.txt)
  constexpr int O3 = 3;
  switch (a.LIST16) {  // >= keep + 4 >= 7; split-candidate plans keep the instances that fit
    case 8: MEPOL_SEL16(8, 3); break;
    case 16: MEPOL_SEL16(16, O3); break;
    case 20: MEPOL_SEL16(20, O3); break;
    case 22: MEPOL_SEL16(22, O3); break;
    case 24: MEPOL_SEL16(24, O3); break;
    case 32: MEPOL_SEL16(32, 1); break;
    default:
      if constexpr (NH == 1 || KS16 <= 2) MEPOL_SEL16(40, 1);
      break;
  }
#undef MEPOL_SEL16
}

template <int KS16>
void launch_select(const SelectArgs& a, hipStream_t st) {
  if (a.seed && a.probe) {
    if (a.nh == 2)
      launch_probe16<KS16, 2>(a, st);
    else
      launch_probe16<KS16, 1>(a, st);
  }
  if (a.nh == 2)
    launch_select16_ks<KS16, 2>(a, st);
  else
    launch_select16_ks<KS16, 1>(a, st);
}

}  // namespace knn
}  // namespace mepol
