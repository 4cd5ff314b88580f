// DROPPED (round 6, measured slower): the k-NN select with TWO query tiles per wave.  Each
// 1-KB candidate fragment feeds two MFMA chains (query tiles A and B); v_permlane32_swap
// exchanges A's upper k-half rows with B's lower ones so that every lane owns one whole query
// and one list of LQ entries (two query tiles at the list registers of one).  Bit-exact (all
// 90 k-NN GPU tests passed with it as the default), but at C3 the call took 6.51 ms
// (occupancy 3, no accumulator pipelining) / 5.95 ms (occupancy 2, pipelined) against 5.11 ms
// for the one-tile kernel: the hit path (16 swaps + 8 row groups per hit tile) runs on nearly
// every tile once 64 queries share one ballot (profiles/r6/knn/qt2_dropped.txt).  It was wired
// through SelectArgs.qt2 and a plan with split lists of LQ per query (refine's list_len = LQ).
// Kept for the record; not built.
#include "../../mepol_amd/csrc/knn_select.hpp"

namespace mepol {
namespace knn {

// ---------------------------------------------------------------------------------------
// Two query tiles per wave (round 6; candidate-hi plans with <= 3 k-steps, k + 1 < LQ).
// The floor of the one-tile kernel above is its fragment traffic: every wave streams 2 KB per
// 32 x 32 tile pair through the texture path (tools/variants/floor_probe.hip: loads + MFMA +
// min tree 3.6 ms at C3, 2.9 ms with two query tiles sharing each fragment).  Here each
// fragment feeds two MFMA chains, query tiles A (queries 64 qp .. +31) and B (+32 .. +63).
// Lane l holds, for column c = l & 31, the k-half h = l >> 5 rows of A's query c and of B's
// query c; v_permlane32_swap exchanges A's upper half with B's lower half, after which lane
// l < 32 holds all 32 rows of A's query l and lane l >= 32 all 32 rows of B's query l - 32.  So
// every lane owns ONE query with ONE list of LQ entries (no half lists, no keep bound): two
// query tiles cost the list registers of one.  The fast path (no lane below its bound) gates
// on the unswapped accumulators against both queries' bounds of the column (the partner
// lane's bound is kept in thr_o); only a hit tile pays the 16 swaps.  Lists go out as one
// list of LQ per (query, range): refine reads split lists of LQ.
// ---------------------------------------------------------------------------------------
constexpr int kGrpCapQ2 = 10;

template <int LIST>
__device__ __forceinline__ void flush_groups_q2(float (&ld)[LIST], int (&li)[LIST], float& thr,
                                                float& thr_o, int& cnt, const f32x4 (*gv)[64],
                                                const int (*gt)[64], int l, float thr0) {
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
      const int i = v0 == x ? 0 : (v1 == x ? 1 : (v2 == x ? 2 : 3));
      if (x < thr) {
        list_insert<LIST>(ld, li, x, tag + i);
        thr = fminf(thr, ld[LIST - 1]);
      }
      v0 = i == 0 ? INFINITY : v0;
      v1 = i == 1 ? INFINITY : v1;
      v2 = i == 2 ? INFINITY : v2;
      v3 = i == 3 ? INFINITY : v3;
    }
  }
  cnt = 0;
  thr = fminf(thr0, fminf(thr, ld[LIST - 1]));
  thr_o = __shfl_xor(thr, 32, kWave);
}

#ifndef MEPOL_Q2_OCC
#define MEPOL_Q2_OCC 3
#endif
#ifndef MEPOL_Q2_PIPE
#define MEPOL_Q2_PIPE 0
#endif
template <int KS16, int LQ>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MEPOL_Q2_OCC))) void select16q2_kernel(
    const _Float16* __restrict__ apack, const float* __restrict__ query, int64_t nq, int d,
    int64_t nct, int split, int64_t tiles_per_split, const unsigned* __restrict__ scal,
    float* __restrict__ out_v, int* __restrict__ out_i, int* __restrict__ seed) {
  __shared__ f32x4 gbv[4][kGrpCapQ2][64];
  __shared__ int gbt[4][kGrpCapQ2][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  const int sp = (int)blockIdx.y;
  const int64_t qtA = ((int64_t)blockIdx.x * 4 + w) * 2;  // query tiles qtA (A), qtA + 1 (B)
  if (qtA * 32 >= nq || (scal[4] | scal[5])) return;       // wave-uniform
  const int h = l >> 5, c = l & 31;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);
  f16x8 bA[KS16], bB[KS16], lo[KS16];
  query_frags<KS16>(query, qtA * 32 + c, nq, d, sg, h, bA, lo);
  query_frags<KS16>(query, qtA * 32 + 32 + c, nq, d, sg, h, bB, lo);
  // the lane's own query after the swap
  const int64_t q = qtA * 32 + l;
  const bool qvalid = q < nq;

  float ld[LQ];
  int li[LQ];
#pragma unroll
  for (int j = 0; j < LQ; ++j) {
    ld[j] = INFINITY;
    li[j] = -1;
  }
  float thr0 = INFINITY;  // seeds: select16_kernel's comment
  if (seed && qvalid)
    thr0 = order_key_float(__hip_atomic_load(seed + q, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM));
  float thr = thr0;
  float thr_o = __shfl_xor(thr, 32, kWave);  // the bound of the other query of this column
  int cnt = 0;
  f32x4(*gv)[64] = gbv[w];
  int(*gt)[64] = gbt[w];

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);
  constexpr int NV = KS16;
  constexpr int NB = 3;
  const f32x4* abase = reinterpret_cast<const f32x4*>(apack) + l;
  f32x4 Bf[NB][NV];
  auto load = [&](f32x4 (&A)[NV], int64_t t) {
    const f32x4* p = abase + t * 64 * NV;
#pragma unroll
    for (int v = 0; v < NV; ++v) A[v] = p[v * 64];
  };
  struct Acc {
    f32x16 a, b;
  };
  auto chain = [&](const f32x4 (&A)[NV]) -> Acc {
    Acc r;
    r.a = f32x16{};
    r.b = f32x16{};
#pragma unroll
    for (int s = 0; s < KS16; ++s) {
      const f16x8 ah = __builtin_bit_cast(f16x8, A[s]);
      r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bA[s], r.a, 0, 0, 0);
      r.b = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bB[s], r.b, 0, 0, 0);
    }
    return r;
  };
  auto add_groups = [&](const f32x16& x, int tb) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float gm = fminf(fminf(x[4 * g], x[4 * g + 1]), fminf(x[4 * g + 2], x[4 * g + 3]));
      if (gm < thr) {
        gv[cnt][l] = f32x4{x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]};
        gt[cnt][l] = tb + 8 * g;
        cnt += 1;
      }
    }
  };
  auto process = [&](Acc x, int64_t t) {
    float mA = x.a[0], mB = x.b[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) {
      mA = fminf(mA, x.a[r]);
      mB = fminf(mB, x.b[r]);
    }
    const float tA = h ? thr_o : thr, tB = h ? thr : thr_o;
    if (__ballot(mA < tA || mB < tB)) {
      // lane l < 32: A rows (h = 0) stay, gets A rows (h = 1) from lane l + 32; lane l >= 32:
      // gets B rows (h = 0) from lane l - 32, B rows (h = 1) stay
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(x.a[r]),
                                                         __float_as_uint(x.b[r]), false, false);
        x.a[r] = __uint_as_float(sw[0]);
        x.b[r] = __uint_as_float(sw[1]);
      }
      const int tb = (int)(t * 32);
      add_groups(x.a, tb);  // rows 8 g + i
      if (__ballot(cnt > kGrpCapQ2 - 4))
        flush_groups_q2<LQ>(ld, li, thr, thr_o, cnt, gv, gt, l, thr0);
      add_groups(x.b, tb + 4);  // rows 8 g + 4 + i
      if (__ballot(cnt > kGrpCapQ2 - 4))
        flush_groups_q2<LQ>(ld, li, thr, thr_o, cnt, gv, gt, l, thr0);
    }
  };
  Acc accP;
  auto step = [&](const f32x4 (&A)[NV], int64_t t, bool prev) {
    const Acc acc = chain(A);
    if constexpr (MEPOL_Q2_PIPE) {
      if (prev) process(accP, t - 1);
      accP = acc;
    } else {
      process(acc, t);
    }
  };
  if (t0 < t1) {
    const int64_t tl = t1 - 1;
#pragma unroll
    for (int b = 0; b < NB - 1; ++b) load(Bf[b], min(t0 + b, tl));
    int64_t t = t0;
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
    for (int b = 1; b < NB; ++b)
      if (t < t1) step_at(b % NB, true);
    if constexpr (MEPOL_Q2_PIPE) process(accP, t - 1);
  }
  flush_groups_q2<LQ>(ld, li, thr, thr_o, cnt, gv, gt, l, thr0);
  if (seed && qvalid)
    __hip_atomic_fetch_min(seed + q, float_order_key(thr), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  if (qvalid) {
    const float bound = fminf(ld[LQ - 1], thr);
    const int64_t o = (q * split + sp) * LQ;
#pragma unroll
    for (int j = 0; j < LQ - 1; ++j) {
      out_v[o + j] = ld[j] * inv_s2;
      out_i[o + j] = li[j];
    }
    out_v[o + LQ - 1] = bound * inv_s2;
    out_i[o + LQ - 1] = (bound < ld[LQ - 1]) ? -1 : li[LQ - 1];
  }
}

template <int KS16>
static void launch_select16q2(const SelectArgs& a, hipStream_t st) {
  const dim3 g((unsigned)((a.nqt + 7) / 8), (unsigned)a.split);
#define MEPOL_SELQ2(L)                                                                      \
  hipLaunchKernelGGL((select16q2_kernel<KS16, L>), g, dim3(256), 0, st, a.apack, a.query, a.nq, \
                     a.d, a.nct, a.split, a.tiles_per_split, a.scal, a.out_v, a.out_i, a.seed)
  switch (a.LIST16) {
    case 16: MEPOL_SELQ2(16); break;
    case 24: MEPOL_SELQ2(24); break;
    default: MEPOL_SELQ2(32); break;
  }
#undef MEPOL_SELQ2
}


}  // namespace knn
}  // namespace mepol
