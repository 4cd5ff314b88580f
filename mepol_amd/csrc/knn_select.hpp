// The k-NN selection kernels (step 2 of knn.hip's pipeline), built once per k-step count by
// knn_select_ks{1..4}.hip.
#pragma once
#include "knn_common.hpp"

namespace mepol {
namespace knn {

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
// OCC = 3: __launch_bounds__(256, 3) caps the kernel at 168 VGPRs (3 waves per SIMD) for the
// short-list instances (a few spilled dwords, on the insertion path only).
template <int KS16, int LIST, int NH, int OCC, int GATE>
__global__ __launch_bounds__(256, OCC) void select16_kernel(const _Float16* __restrict__ apack,
                                                       const float* __restrict__ query,
                                                       int64_t nq, int d, int64_t nct, int split,
                                                       int64_t tiles_per_split, int keep,
                                                       const unsigned* __restrict__ scal,
                                                       float* __restrict__ out_v,
                                                       int* __restrict__ out_i,
                                                       int* __restrict__ seed) {
  // per-lane insertion buffer: (value, index bits) pairs, one 8-byte LDS access per entry
  __shared__ float2 sbuf[4][kBufCap][64];
  const int w = threadIdx.x >> 6;
  const int l = threadIdx.x & 63;
  // XCD-aware block mapping: workgroups go round-robin over the 8 XCDs by linear id, so with
  // sp = id % split (split a multiple of 8) every XCD only ever reads the candidate ranges
  // sp = xcd (mod 8), which then stay resident in that XCD's 4 MB L2.  Any other split (2 at
  // C3) keeps the split-major order: the blocks in flight then all read one candidate range.
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const bool xcd_map = (split & 7) == 0;
  const int sp = xcd_map ? (int)(lin % split) : (int)blockIdx.y;
  const int64_t qt = (xcd_map ? lin / split : (int64_t)blockIdx.x) * 4 + w;
  if (qt * 32 >= nq || (scal[4] | scal[5])) return;  // wave-uniform (rejected input: knn.hip)
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
  // Retire the B-operand loads here and launder the registers, so no compiler-tracked load is
  // pending inside the tile loop (otherwise its waitcnt pass drains vmcnt(0) every iteration).
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s = 0; s < KS16; ++s) {
    f32x4 x = __builtin_bit_cast(f32x4, bhi[s]);
    f32x4 y = __builtin_bit_cast(f32x4, blo[s]);
    asm volatile("" : "+v"(x), "+v"(y));
    bhi[s] = __builtin_bit_cast(f16x8, x);
    blo[s] = __builtin_bit_cast(f16x8, y);
  }

  float ld[LIST];
  int li[LIST];
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    ld[j] = INFINITY;
    li[j] = -1;
  }
  // Seed of the prune bound: the tightest bound a range of this query already finished with
  // (the grid runs split-major, so range 0's blocks are mostly done when range 1's start).  Any
  // value is sound -- a lane only claims what its own scan rejected against its own bound, and
  // refine certifies against the reported bounds -- and every published bound has >= 2 keep
  // candidates of its range at or below it, so it costs no certification.  It skips most of the
  // list warm-up, where the bulk of the insertions happen.  System scope: the load and the
  // publishing atomic below go past the XCD's own (non-coherent) L2.
  float thr0 = INFINITY;
  if (seed && qvalid)
    thr0 = order_key_float(
        __hip_atomic_load(seed + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  float thr = thr0;
  int cnt = 0;

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);

  // Fragment buffers in registers: tile t's MFMAs run while tile t-1's threshold work executes
  // and the next tiles' loads are in flight; a buffer is refilled only after the chain that
  // read it has completed.  Loads are inline asm with hand-counted waits (NV per tile; no other
  // vector-memory op in the loop).  Three buffers, two where a 4-k-step tile and long lists
  // would otherwise reach the 256-VGPR cap (at the cap the asm-load buffers are not safe from
  // register copies).
  constexpr int NV = NH * KS16;  // dwordx4 per lane per tile: one per (k-step, half)
  // query lo half: split-candidate plans and 4-k-step plans (make_plan's bound covers the rest)
  constexpr bool kQueryLo = NH == 2 || KS16 >= 4;
  constexpr int NB = NH == 2 ? (KS16 >= 4 ? 2 : 3) : ((KS16 >= 4 && LIST > 32) ? 2 : 3);
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + l;
  f32x4 Bf[NB][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      f32x4 x;
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(x) : "v"(p + v * 64) : "memory");
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
  auto process = [&](f32x16 acc, int64_t t) {
    // min over the 4 row groups (rows 4g..4g+3), then over the groups
    float gm[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      gm[g] = fminf(fminf(acc[4 * g], acc[4 * g + 1]), fminf(acc[4 * g + 2], acc[4 * g + 3]));
    const float m = fminf(fminf(gm[0], gm[1]), fminf(gm[2], gm[3]));
    if (__ballot(m < thr)) {
      const int base = (int)(t * 32);
      if constexpr (GATE == 5) {
        // row groups gated as below, the rows of a hit group branch-free: every lane of the
        // group writes its value at its cursor and advances the cursor only when the value is
        // under its bound (a later write overwrites a rejected one).  The cursor enters a tile
        // at <= kBufCap - 16 (flush condition below), so the write index stays < kBufCap.
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (gm[g] < thr) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              sbuf[w][cnt][l] = make_float2(acc[r], __int_as_float(base + acc_row(r, l)));
              cnt += acc[r] < thr ? 1 : 0;
            }
          }
        }
      } else if constexpr (GATE == 4) {
        // hierarchical gating: a row group is skipped by the whole wave unless some lane has a
        // value under its bound there (4 group tests + 4 row tests per hit group instead of 16
        // row tests per hit tile)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (gm[g] < thr) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int r = 4 * g + i;
              if (acc[r] < thr) {
                sbuf[w][cnt][l] = make_float2(acc[r], __int_as_float(base + acc_row(r, l)));
                ++cnt;
              }
            }
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          if (acc[r] < thr) {
            sbuf[w][cnt][l] = make_float2(acc[r], __int_as_float(base + acc_row(r, l)));
            ++cnt;
          }
        }
      }
      if (__ballot(cnt > kBufCap - 16))
        flush_buffer<LIST>(ld, li, thr, cnt, sbuf[w], l, thr0, keep);
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
  flush_buffer<LIST>(ld, li, thr, cnt, sbuf[w], l, thr0, keep);
  // publish this range's final bound (the same in both lanes of the query)
  if (seed && qvalid && h == 0)
    __hip_atomic_fetch_min(seed + q, float_order_key(thr), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);

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

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
static inline int select_occ3() {
  const char* e = getenv("MEPOL_KNN_OCC3");
  return !(e && e[0] == '0');
}

template <int KS16, int NH, int GATE>
static void launch_select16_gate(const SelectArgs& a, hipStream_t st) {
  const dim3 g((unsigned)((a.nqt + 3) / 4), (unsigned)a.split);
#define MEPOL_SEL16O(L, O)                                                                        \
  hipLaunchKernelGGL((select16_kernel<KS16, L, NH, O, GATE>), g, dim3(256), 0, st, a.apack,      \
                     a.query, a.nq, a.d, a.nct, a.split, a.tiles_per_split, a.keep, a.scal, a.out_v,       \
                     a.out_i, a.seed)
#define MEPOL_SEL16(L) MEPOL_SEL16O(L, 1)
  switch (a.LIST16) {  // >= keep + 4 >= 7; split-candidate plans keep the instances that fit
    case 8: MEPOL_SEL16(8); break;
    case 16: MEPOL_SEL16(16); break;
    case 22:
      if constexpr (NH == 1 && KS16 <= 2) {
        if (select_occ3()) {
          MEPOL_SEL16O(22, 3);
          break;
        }
      }
      MEPOL_SEL16(22);
      break;
    case 24:
      if constexpr (NH == 1 && KS16 <= 2) {
        if (select_occ3()) {
          MEPOL_SEL16O(24, 3);
          break;
        }
      }
      MEPOL_SEL16(24);
      break;
    case 32: MEPOL_SEL16(32); break;
    default:
      if constexpr (NH == 1 || KS16 <= 2) MEPOL_SEL16(40);
      break;
  }
#undef MEPOL_SEL16
#undef MEPOL_SEL16O
}

// MEPOL_KNN_GATE (A/B probe): 1 = round 3's per-row gating of a hit tile, 4 = row groups with
// a branch per row, 5 (default) = row groups with branch-free rows.
static int select_gate() {
  static const int v = [] {
    const char* e = getenv("MEPOL_KNN_GATE");
    return (e && e[0] == '1') ? 1 : (e && e[0] == '4') ? 4 : 5;
  }();
  return v;
}

template <int KS16, int NH>
static void launch_select16_ks(const SelectArgs& a, hipStream_t st) {
  if constexpr (NH == 1) {
    if (select_gate() == 5) {
      launch_select16_gate<KS16, NH, 5>(a, st);
      return;
    }
    if (select_gate() == 4) {
      launch_select16_gate<KS16, NH, 4>(a, st);
      return;
    }
  }
  launch_select16_gate<KS16, NH, 1>(a, st);
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
