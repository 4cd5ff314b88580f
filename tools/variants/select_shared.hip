// DROPPED (round 5, measured slower): the k-NN select with the candidate fragments shared by
// the workgroup's four waves through an LDS ring filled by LDS-DMA, one barrier per interval.
// It cut the texture-path traffic 3x (TA_BUSY 1.63e9 -> 0.51e9, TD_BUSY 2.14e9 -> 1.01e9) but
// the waves waited on each other at the barriers (SQ_WAIT_ANY 1.84e9 -> 5.47e9): select
// 4.8 -> 6.8 ms at C3 (profiles/r5/knn/shared_select_dropped.txt).  Kept for the record; not
// built.  It used the product's LaneList / list helpers (mepol_amd/csrc/knn_select.hpp) and a
// per-lane (value, index) insertion buffer flushed by flush_buffer<LIST, CAP>.
#include "../../mepol_amd/csrc/knn_select.hpp"

namespace mepol {
namespace knn {
// ---------------------------------------------------------------------------------------
// select16s_kernel: the same selection with the candidate fragments shared by the workgroup's
// four waves through an LDS ring.  The register-streamed kernel above loads every fragment into
// every wave (1 KB per k-step, tile and wave): at C3 the texture path ran 84 % busy (TD) and
// the fragment loads alone took 3.3 of its 4.8 ms (profiles/r5/knn/).  Here each fragment is
// fetched once per workgroup by LDS-DMA (global_load_lds_dwordx4, 1 KB per wave-instruction,
// the waves taking turns) and read by the four waves with ds_read_b128.  The ring is two
// stages of R tiles: interval i's tiles are read from stage i & 1 while interval i + 1's DMA
// fills the other stage, issued right after the barrier that opens interval i (that stage was
// last read in interval i - 1, which every wave has finished at the barrier); each wave waits
// for its own DMA (vmcnt(0), one interval after issue) before that barrier.  One barrier per
// R tiles.  Lists, bounds, seeds and outputs are the register kernel's.
// ---------------------------------------------------------------------------------------
template <int KS16, int LIST, int NH, int R, int CAP, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) void select16s_kernel(
    const _Float16* __restrict__ apack, const float* __restrict__ query, int64_t nq, int d,
    int64_t nct, int split, int64_t tiles_per_split, int keep, const unsigned* __restrict__ scal,
    float* __restrict__ out_v, int* __restrict__ out_i, int* __restrict__ seed) {
  constexpr int NV = NH * KS16;  // 1-KB fragments per tile
  constexpr int NF = R * NV;     // fragments per interval
  // two stages as two objects, so the compiler's wait insertion sees that the DMA into one
  // stage does not alias the reads of the other (one array with a runtime stage index made it
  // wait for the just-issued DMA before the first read of every interval)
  __shared__ f32x4 ringA[NF][64];
  __shared__ f32x4 ringB[NF][64];
  __shared__ float2 sbuf[4][CAP][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  const int64_t lin = (int64_t)blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  const bool xcd_map = (split & 7) == 0;
  const int sp = xcd_map ? (int)(lin % split) : (int)blockIdx.y;
  const int64_t qt0 = (xcd_map ? lin / split : (int64_t)blockIdx.x) * 4 + w;
  if (scal[4] | scal[5]) return;  // rejected input: uniform over the workgroup
  // waves past the last query tile keep loading and meeting the barriers, and select nothing
  const bool active = qt0 * 32 < nq;  // wave-uniform
  const int h = l >> 5;
  const float sg = knn_scale(scal);
  const float inv_s2 = 1.f / (sg * sg);
  constexpr bool kQueryLo = NH == 2 || KS16 >= 4;

  f16x8 bhi[KS16], blo[KS16];
  const int64_t q = qt0 * 32 + (l & 31);
  const bool qvalid = q < nq;
  {
    const float* qrow = query + min(q, nq - 1) * d;
#pragma unroll
    for (int s = 0; s < KS16; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int f = 16 * s + 8 * h + j;
        const float x = qrow[min(f, d - 1)];
        const float v = ((f < d ? sg : 0.f) * x + (f == d ? 1.f : 0.f)) * (qvalid ? 1.f : 0.f);
        _Float16 a, b;
        split_f16(v, a, b);
        bhi[s][j] = a;
        blo[s][j] = b;
      }
  }
  LaneList<LIST> S;
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    S.ld[j] = INFINITY;
    S.li[j] = -1;
  }
  S.thr0 = INFINITY;
  if (seed && qvalid)
    S.thr0 = order_key_float(
        __hip_atomic_load(seed + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  S.thr = S.thr0;
  S.cnt = 0;
  float2(*buf)[64] = sbuf[w];

  const int64_t t0 = (int64_t)sp * tiles_per_split;
  const int64_t t1 = min(nct, t0 + tiles_per_split);
  const int64_t tl = t1 - 1;
  const f32x4* asrc = reinterpret_cast<const f32x4*>(apack) + l;

  // DMA of interval ii into stage ii & 1: fragment f = (tile j of the interval, part v); wave w
  // issues f = w, w + 4, ...  (tiles past the range re-read the last one and are not used)
  auto issue = [&](f32x4 (&dst)[NF][64], int64_t ii) __attribute__((always_inline)) {
#pragma unroll
    for (int f = 0; f < NF; f += 4) {
      if (f + w < NF) {  // wave-uniform
        const int ff = f + w;
        const int64_t tt = min(t0 + ii * R + ff / NV, tl);
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(asrc + (tt * NV + ff % NV) * 64),
            (__attribute__((address_space(3))) void*)&dst[ff][0], 16, 0, 0);
      }
    }
  };
  auto chain = [&](const f32x4 (&A)[NV]) __attribute__((always_inline)) -> f32x16 {
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
  auto process = [&](const f32x16& acc, int64_t t) __attribute__((always_inline)) {
    float gm[4];
#pragma unroll
    for (int g = 0; g < 4; ++g)
      gm[g] = fminf(fminf(acc[4 * g], acc[4 * g + 1]), fminf(acc[4 * g + 2], acc[4 * g + 3]));
    const float m = fminf(fminf(gm[0], gm[1]), fminf(gm[2], gm[3]));
    if (__ballot(m < S.thr)) {
      const int base = (int)(t * 32) + 4 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (gm[g] < S.thr) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = 4 * g + i;
            buf[S.cnt][l] = make_float2(acc[r], __int_as_float(base + ((r & 3) + 8 * (r >> 2))));
            S.cnt += acc[r] < S.thr ? 1 : 0;
          }
        }
        // a pair of row groups adds <= 8 entries: the cursor stays < CAP
        if ((g & 1) && __ballot(S.cnt > CAP - 8))
          flush_buffer<LIST, CAP>(S.ld, S.li, S.thr, S.cnt, buf, l, S.thr0, keep);
      }
    }
  };

  const int64_t nint = (t1 - t0 + R - 1) / R;
  f32x16 accP = {};
  bool have = false;
  int64_t tp = 0;
  // interval ii: every wave's DMA of it has landed (own vmcnt(0) + the barrier), the DMA of
  // ii + 1 goes into the other stage, then the R tiles are read from `cur`
  auto interval = [&](f32x4 (&cur)[NF][64], f32x4 (&nxt)[NF][64], int64_t ii)
                      __attribute__((always_inline)) {
    __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's DMA into `cur`
    __syncthreads();
    if (ii + 1 < nint) issue(nxt, ii + 1);
    if (!active) return;
    const int nj = (int)min<int64_t>(R, t1 - (t0 + ii * R));
    f32x4 A[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) A[v] = cur[v][l];
    // not unrolled: one copy of the threshold / insertion code per stage (instruction cache)
#pragma nounroll
    for (int j = 0; j < nj; ++j) {
      f32x4 An[NV];
      const int jn = min(j + 1, R - 1);  // the last tile re-reads itself (unused)
#pragma unroll
      for (int v = 0; v < NV; ++v) An[v] = cur[jn * NV + v][l];
      const f32x16 acc = chain(A);
#if MEPOL_SEL_PROBE == 1
      S.cnt += acc[0] < -1e30f ? 1 : 0;  // keep the MFMA live
#else
      if (have) process(accP, tp);
#endif
      accP = acc;
      tp = t0 + ii * R + j;
      have = true;
#pragma unroll
      for (int v = 0; v < NV; ++v) A[v] = An[v];
    }
  };
  if (t0 < t1) issue(ringA, 0);
  for (int64_t ii = 0; ii < nint; ii += 2) {
    interval(ringA, ringB, ii);
    if (ii + 1 < nint) interval(ringB, ringA, ii + 1);
  }
  if (!active) return;
  if (have) process(accP, tp);
  flush_buffer<LIST, CAP>(S.ld, S.li, S.thr, S.cnt, buf, l, S.thr0, keep);
  if (seed && qvalid && h == 0)
    __hip_atomic_fetch_min(seed + q, float_order_key(S.thr), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
  if (qvalid) {
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

}  // namespace knn
}  // namespace mepol
