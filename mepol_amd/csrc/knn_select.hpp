// The k-NN selection kernels (step 2 of knn.hip's pipeline), built once per k-step count by
// knn_select_ks{1..4}.hip.
#pragma once
#include "knn_common.hpp"

namespace mepol {
namespace knn {

// Per-query state of a lane: its sorted top-LIST list (values ascending), the prune bound, the
// seed it started from and the fill of its LDS insertion buffer.
template <int LIST>
struct LaneList {
  float ld[LIST];
  int li[LIST];
  float thr, thr0;
  int cnt;
};

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
// QT query tiles of 32 per wave (one lane = one query column of each).  The candidate
// fragments are the kernel's dominant traffic (1 KB per k-step, half and tile, from L2 into
// every wave that reads it): at C3 the loads alone held the round-4 kernel (QT = 1) at 3.34 of its
// 4.78 ms, at ~45 B/clk per CU (profiles/r5/knn/select_breakdown.txt).  With QT = 2 each loaded
// fragment feeds two MFMA chains, halving the bytes per query-candidate pair; the waves stay
// independent (sharing a tile between waves through LDS needs a barrier per tile, and the
// barrier made every wave wait out the others' list insertions: 7.2 ms,
// profiles/r5/knn/lds_ring_dropped.txt).  Waves per workgroup WPB = 4 / QT: a workgroup covers
// 4 query tiles either way.
// OCC: waves per SIMD the VGPR budget is cut for (__launch_bounds__).
template <int KS16, int LIST, int NH, int QT, int OCC>
__global__ __launch_bounds__(256 / QT) __attribute__((amdgpu_waves_per_eu(OCC))) void select16_kernel(
    const _Float16* __restrict__ apack, const float* __restrict__ query, int64_t nq, int d,
    int64_t nct, int split, int64_t tiles_per_split, int keep, const unsigned* __restrict__ scal,
    float* __restrict__ out_v, int* __restrict__ out_i, int* __restrict__ seed) {
  constexpr int WPB = 4 / QT;
  // per-lane insertion buffers: (value, index bits) pairs, one 8-byte LDS access per entry
  __shared__ float2 sbuf[WPB][QT][kBufCap][64];
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  // XCD-aware block mapping: workgroups go round-robin over the 8 XCDs by linear id, so with
  // sp = id % split (split a multiple of 8) every XCD only ever reads the candidate ranges
  // sp = xcd (mod 8), which then stay resident in that XCD's 4 MB L2.  Any other split (2 at
  // C3) keeps the split-major order: the blocks in flight then all read one candidate range.
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const bool xcd_map = (split & 7) == 0;
  const int sp = xcd_map ? (int)(lin % split) : (int)blockIdx.y;
  const int64_t qt0 = ((xcd_map ? lin / split : (int64_t)blockIdx.x) * WPB + w) * QT;
  if (qt0 * 32 >= nq || (scal[4] | scal[5])) return;  // wave-uniform (rejected input: knn.hip)
  const int h = l >> 5;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);  // exact: sigma is a power of two
  constexpr bool kQueryLo = NH == 2 || KS16 >= 4;  // make_plan's bound covers the rest

  // B operands (queries): B[k = 16 s + 8h + j][col = l&31] = sigma q_f (f<d), 1 (f==d), 0.
  // Unconditional loads at clamped addresses (a load under a per-element condition makes hipcc
  // wait for each one in turn).
  f16x8 bhi[QT][KS16], blo[QT][KS16];
  int64_t q[QT];
  bool qvalid[QT];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
    q[u] = (qt0 + u) * 32 + (l & 31);
    qvalid[u] = q[u] < nq;
    const float* qrow = query + min(q[u], nq - 1) * d;
#pragma unroll
    for (int s = 0; s < KS16; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * s + 8 * h + j;
        const float x = qrow[min(f, d - 1)];  // finite (validated): x * 0 = 0
        const float v = ((f < d ? sg : 0.f) * x + (f == d ? 1.f : 0.f)) * (qvalid[u] ? 1.f : 0.f);
        _Float16 a, b;
        split_f16(v, a, b);
        bhi[u][s][j] = a;
        blo[u][s][j] = b;
      }
  }

  LaneList<LIST> L[QT];
#pragma unroll
  for (int u = 0; u < QT; ++u) {
#pragma unroll
    for (int j = 0; j < LIST; ++j) {
      L[u].ld[j] = INFINITY;
      L[u].li[j] = -1;
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
    L[u].thr0 = INFINITY;
    if (seed && qvalid[u])
      L[u].thr0 = order_key_float(
          __hip_atomic_load(seed + q[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
    L[u].thr = L[u].thr0;
    L[u].cnt = 0;
  }

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  // Fragment ring in registers: tile t's MFMAs run while the next tiles' loads are in flight; a
  // buffer is refilled only after the chains that read it were issued.  Plain loads: hipcc
  // counts the waits (each step waits for the oldest tile in flight only).
  constexpr int NV = NH * KS16;  // dwordx4 per lane per tile: one per (k-step, half)
#ifndef MEPOL_SEL_NB
#define MEPOL_SEL_NB 3
#endif
  constexpr int NB = MEPOL_SEL_NB;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + l;
  f32x4 Bf[NB][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) A[v] = p[v * 64];
  };
  auto chain = [&](const f32x4 (&A)[NV], int u) -> f32x16 {
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < KS16; ++s) {
      const f16x8 ah = __builtin_bit_cast(f16x8, A[NH * s]);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bhi[u][s], acc, 0, 0, 0);
      if constexpr (kQueryLo)
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, blo[u][s], acc, 0, 0, 0);
      if constexpr (NH == 2) {
        const f16x8 al = __builtin_bit_cast(f16x8, A[2 * s + 1]);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bhi[u][s], acc, 0, 0, 0);
      }
    }
    return acc;
  };
  // (the per-query calls below name L[0] / L[1] with constant indices: a runtime index into L
  // would put the lists in scratch memory)
  auto process = [&](const f32x16& acc, int64_t t, LaneList<LIST>& S, float2 (*buf)[64]) {
    // min over the 4 row groups (rows 4g..4g+3), then over the groups
    float gm[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      gm[g] = fminf(fminf(acc[4 * g], acc[4 * g + 1]), fminf(acc[4 * g + 2], acc[4 * g + 3]));
    const float m = fminf(fminf(gm[0], gm[1]), fminf(gm[2], gm[3]));
    if (__ballot(m < S.thr)) {
      const int base = (int)(t * 32);
      // Row groups are skipped by the whole wave unless some lane has a value under its bound
      // there; the rows of a hit group are branch-free: every lane writes its value at its
      // cursor and advances the cursor only when the value is under its bound (a later write
      // overwrites a rejected one).  The cursor enters a tile at <= kBufCap - 16 (flush
      // condition below), so the write index stays < kBufCap.
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (gm[g] < S.thr) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * g + i;
            buf[S.cnt][l] = make_float2(acc[r], __int_as_float(base + acc_row(r, l)));
            S.cnt += acc[r] < S.thr ? 1 : 0;
          }
        }
      }
      if (__ballot(S.cnt > kBufCap - 16))
        flush_buffer<LIST>(S.ld, S.li, S.thr, S.cnt, buf, l, S.thr0, keep);
    }
  };
  // Every chain's MFMA latency hides under threshold work issued after it.  QT = 1: tile t's
  // chain, then tile t-1's accumulators.  QT = 2 (one carried accumulator instead of two):
  // chain (t, 0); process (t-1, 1); chain (t, 1); process (t, 0); carry (t, 1).
  f32x16 accP;
  auto step = [&](const f32x4 (&A)[NV], int64_t t, bool prev) {
    const f32x16 acc0 = chain(A, 0);
    if constexpr (QT == 2) {
      if (prev) process(accP, t - 1, L[QT - 1], sbuf[w][QT - 1]);
      accP = chain(A, QT - 1);
      process(acc0, t, L[0], sbuf[w][0]);
    } else {
      if (prev) process(accP, t - 1, L[0], sbuf[w][0]);
      accP = acc0;
    }
  };
  if (t0 < t1) {
    const int64_t tl = t1 - 1;
#pragma unroll
    for (int b = 0; b < NB - 1; ++b) load(Bf[b], min(t0 + b, tl));
    int64_t t = t0;
    // steady state, unrolled by NB so buffer indices are compile-time: tile t is in
    // Bf[(t - t0) % NB]; the buffer of tile t - 1 (its chains issued) takes tile t + NB - 1 (the
    // refills of the last tiles re-read tile t1 - 1).
    auto step_at = [&](int cur, bool prev) {
      load(Bf[(cur + NB - 1) % NB], min(t + NB - 1, tl));
      step(Bf[cur], t, prev);
      ++t;
    };
    step_at(0, false);
    // t0 + 1 onward: tile t in Bf[(t - t0) % NB], rounds of NB starting at buffer 1
#pragma nounroll
    while (t + NB - 1 < t1) {
#pragma unroll
      for (int b = 1; b <= NB; ++b) step_at(b % NB, true);
    }
#pragma unroll
    for (int b = 1; b < NB; ++b)  // remainder (0..NB-1 tiles), same buffer rotation
      if (t < t1) step_at(b % NB, true);
    process(accP, t - 1, L[QT - 1], sbuf[w][QT - 1]);
  }

  auto finish = [&](int u, LaneList<LIST>& S) {
    if ((qt0 + u) * 32 >= nq) return;  // wave-uniform
    flush_buffer<LIST>(S.ld, S.li, S.thr, S.cnt, sbuf[w][u], l, S.thr0, keep);
    // publish this range's final bound (the same in both lanes of the query)
    if (seed && qvalid[u] && h == 0)
      __hip_atomic_fetch_min(seed + q[u], float_order_key(S.thr), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    if (qvalid[u]) {
      // The last slot carries this lane's final bound: every candidate of its range that is not
      // in the list has an approximate value >= min(list last, thr) (rejected against thr, or
      // evicted from the list); a last entry at or above the bound is dropped (idx -1), the
      // bound covers it.  refine takes the min over the query's lanes.
      const float bound = fminf(S.ld[LIST - 1], S.thr);
      const int64_t o = ((q[u] * split + sp) * 2 + h) * LIST;
#pragma unroll
      for (int j = 0; j < LIST - 1; ++j) {
        out_v[o + j] = S.ld[j] * inv_s2;
        out_i[o + j] = S.li[j];
      }
      out_v[o + LIST - 1] = bound * inv_s2;
      out_i[o + LIST - 1] = (bound < S.ld[LIST - 1]) ? -1 : S.li[LIST - 1];
    }
  };
  finish(0, L[0]);
  if constexpr (QT == 2) finish(1, L[QT - 1]);
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
#ifndef MEPOL_SEL_QT
#define MEPOL_SEL_QT 1
#endif
template <int KS16, int NH>
static void launch_select16_ks(const SelectArgs& a, hipStream_t st) {
  const dim3 g((unsigned)((a.nqt + 3) / 4), (unsigned)a.split);
#define MEPOL_SEL16Q(L, QT, O)                                                                   \
  hipLaunchKernelGGL((select16_kernel<KS16, L, NH, QT, O>), g, dim3(256 / QT), 0, st, a.apack,  \
                     a.query, a.nq, a.d, a.nct, a.split, a.tiles_per_split, a.keep, a.scal,     \
                     a.out_v, a.out_i, a.seed)
  // two query tiles per wave where the lists leave room (2 waves per SIMD), one otherwise
#ifndef MEPOL_SEL_OCC1
#define MEPOL_SEL_OCC1 3
#endif
#define MEPOL_SEL16(L) MEPOL_SEL16Q(L, MEPOL_SEL_QT, (MEPOL_SEL_QT == 2 ? 2 : MEPOL_SEL_OCC1))
  switch (a.LIST16) {  // >= keep + 4 >= 7; split-candidate plans keep the instances that fit
    case 8: MEPOL_SEL16(8); break;
    case 16: MEPOL_SEL16(16); break;
    case 22: MEPOL_SEL16(22); break;
    case 24: MEPOL_SEL16(24); break;
    case 32: MEPOL_SEL16Q(32, 1, 1); break;
    default:
      if constexpr (NH == 1 || KS16 <= 2) MEPOL_SEL16Q(40, 1, 1);
      break;
  }
#undef MEPOL_SEL16
#undef MEPOL_SEL16Q
}

template <int KS16>
void launch_select(const SelectArgs& a, hipStream_t st) {
  if (a.nh == 2)
    launch_select16_ks<KS16, 2>(a, st);
  else
    launch_select16_ks<KS16, 1>(a, st);
}

}  // namespace knn
}  // namespace mepol
