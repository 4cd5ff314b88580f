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
// Pipeline (one stream, no allocation; one host sync for the input check):
//   0. norms   : max |c|, max |q| and the NaN / inf / overflow counts (input validation).
//   1. pack    : candidates scaled by a power of two sigma, A = [-2 sigma c, |sigma c|^2]
//                rounded to f16 (the hi half only) in v_mfma_f32_32x32x16_f16 A-fragment
//                order: one 1-KB block per (32-candidate tile, k-step of 16).
//   2. select  : per 32-query tile (one wave) and candidate range, 2 MFMAs per k-step
//                (A_hi x q_hi + A_hi x q_lo, f32 accumulate) give |c|^2 - 2 q.c for 32 x 32
//                pairs; each lane owns one query column and keeps a sorted top-LIST list in
//                VGPRs, fed through a per-lane LDS buffer (insertions paid in batches).
//   3. refine  : per query, merge the 2*split partial lists to the approximate top-64,
//                recompute the distances inside the selection's error band exactly in f64,
//                bitonic-sort by (dist, idx), and certify with a rigorous bound on the f16
//                selection's error that no excluded candidate can enter the top-(k+1).
//                Uncertified queries (near-ties across the boundary, duplicate clusters) are
//                queued.
//   4. exact   : queued queries are answered by an exhaustive f64 scan (no approximation),
//                a handful of queries spread over the whole grid (chunked scan + merge).
#include "knn_common.hpp"

namespace mepol {
namespace knn {

// ---------------------------------------------------------------------------------------
// 0./1. input check, scale and pack
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

// Row blocks of the norms / pack kernels: the rows are read into LDS as one contiguous span
// (one coalesced 256-B access per wave-instruction; a row per lane read straight from HBM would
// touch 64 lines per instruction, d-float stride) and used from there.
constexpr int kStageRows = 128;

// kStageRows rows of X (d floats each) into sx, coalesced, kStageBatch loads in flight per
// thread (a plain copy loop waits for each load before its LDS store).  Returns the rows present.
constexpr int kStageBatch = 8;
__device__ __forceinline__ int stage_rows(const float* __restrict__ X, int64_t n, int d, int64_t r0,
                                          float* sx) {
  const int rows = (int)min<int64_t>(kStageRows, n - r0);
  const int cnt = rows * d;
  const float* src = X + r0 * d;
  const int nt = blockDim.x;
  for (int e0 = threadIdx.x; e0 < cnt; e0 += kStageBatch * nt) {
    float v[kStageBatch];
#pragma unroll
    for (int u = 0; u < kStageBatch; ++u) v[u] = src[min(e0 + u * nt, cnt - 1)];
#pragma unroll
    for (int u = 0; u < kStageBatch; ++u)
      if (e0 + u * nt < cnt) sx[e0 + u * nt] = v[u];
  }
  __syncthreads();
  return rows;
}

// out_bits2 (nullable): a second max slot fed from the same rows (queries == candidates: the
// self k-NN of mepol.py:190-192 needs one pass, not two).  Launched with 256 threads per block
// (all of them stage rows; threads < kStageRows then reduce one row each; grid-stride over row
// blocks) and kStageRows * d floats of dynamic LDS.  One atomic per block and slot, and few
// blocks: the max lands on one address from every block, and those device-scope atomics
// serialise (1563 blocks took ~42 us at 200k rows, where staging the rows takes ~10).
constexpr int kNormsBlocks = 256;
constexpr int kNormsThreads = 256;
__global__ __launch_bounds__(kNormsThreads) void norms_kernel(const float* __restrict__ X, int64_t n,
                                                           int d, unsigned* __restrict__ out_bits,
                                                           unsigned* __restrict__ bad,
                                                           unsigned* __restrict__ out_bits2) {
  extern __shared__ float sx[];
  __shared__ float s_nrm[kNormsThreads / 64];
  __shared__ unsigned s_bad[2];
  if (threadIdx.x == 0) s_bad[0] = s_bad[1] = 0u;
  float nrm = 0.f;
  unsigned nonfinite_rows = 0, overflow_rows = 0;
  for (int64_t r0 = (int64_t)blockIdx.x * kStageRows; r0 < n; r0 += (int64_t)gridDim.x * kStageRows) {
    __syncthreads();  // the previous step's LDS reads are done
    const int rows = stage_rows(X, n, d, r0, sx);
    if ((int)threadIdx.x < rows) {
      const float* x = sx + threadIdx.x * d;
      float s2 = 0.f;
      unsigned mag = 0;  // max |x_f| bit pattern: integer ops, no float compare to fold
      for (int f = 0; f < d; ++f) {
        const float v = x[f];
        mag = max(mag, __float_as_uint(v) & 0x7fffffffu);
        s2 = fmaf(v, v, s2);
      }
      const bool nonfinite = nonfinite_bits(__uint_as_float(mag));
      const bool overflow = !nonfinite && nonfinite_bits(s2);
      nonfinite_rows += nonfinite;
      overflow_rows += overflow;
      if (!nonfinite && !overflow) nrm = fmaxf(nrm, sqrtf(s2));
    }
  }
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) nrm = fmaxf(nrm, __shfl_xor(nrm, m, kWave));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) s_nrm[w] = nrm;
  __syncthreads();
  if (nonfinite_rows) atomicAdd(&s_bad[0], nonfinite_rows);
  if (overflow_rows) atomicAdd(&s_bad[1], overflow_rows);
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = s_nrm[0];
    for (int i = 1; i < kNormsThreads / 64; ++i) m = fmaxf(m, s_nrm[i]);
    atomicMax(out_bits, __float_as_uint(m));
    if (out_bits2) atomicMax(out_bits2, __float_as_uint(m));
    if (s_bad[0]) atomicAdd(bad, s_bad[0]);
    if (s_bad[1]) atomicAdd(bad + 1, s_bad[1]);
  }
}

// The f16 screen does not run for this input: norms_kernel counted into scal[4] the rows with a
// NaN / inf coordinate (rejected input: the deferred entry point does not stop the stream to
// look, so every later kernel returns at once, the outputs are undefined and the caller raises)
// and into scal[5] the finite rows whose squared norm overflows f32 (valid input that the f16
// scale cannot represent: the screen is skipped and every query takes the exhaustive f64 stage,
// knn_exact.hip).  Only scal[4] is a rejection.
__device__ __forceinline__ bool skip_screen(const unsigned* __restrict__ scal) {
  return (scal[4] | scal[5]) != 0u;
}

// apack16[((t*64 + l)*KS16 + s)*16 + {0..7 hi, 8..15 lo}] = A[i = l&31][k = 16 s + 8 (l>>5) + j]
// of candidate tile t: f<d: -2 sigma x_cf ; f==d: |sigma c|^2 ; else 0.
// apack16[(((t*KS16 + s)*nh + u)*64 + l)*8 + j] = half u of A[i = l&31][k = 16 s + 8 (l>>5) + j]
// of candidate tile t, A = [-2 sigma c, |sigma c|^2, 0...]; u = 0: fl16(A) (hi), u = 1 (nh = 2
// only): fl16(A - hi) (lo).  Each (k-step, half) of a tile is 1 KB, one coalesced dwordx4 per
// lane.  Padding candidates carry a norm above every real value.
// Also writes cpad [n][dp] f32: the candidate rows padded with zeros to dp = a multiple of 32
// floats (128-B aligned): refine's exact-distance gathers then read whole lines with dwordx4.
__global__ __launch_bounds__(256) void pack16_kernel(const float* __restrict__ X, int64_t n, int d,
                                                     int KS16, int nh, int64_t nct,
                                                     _Float16* __restrict__ apack,
                                                     const unsigned* __restrict__ scal,
                                                     float* __restrict__ cpad, int dp) {
  // 4 tiles (kStageRows = 128 candidates) per block of 256 threads, staged through LDS
  extern __shared__ float sx[];
  if (skip_screen(scal)) return;  // block-uniform, before the barrier
  const int64_t c0 = (int64_t)blockIdx.x * kStageRows;
  const int rows = stage_rows(X, n, d, c0, sx);
  // cpad rows of this block: one contiguous span, written with dwordx4 in order
  {
    f32x4* dst = reinterpret_cast<f32x4*>(cpad + c0 * dp);
    const int nv = rows * dp / 4;
    for (int e = threadIdx.x; e < nv; e += blockDim.x) {
      const int r = (4 * e) / dp, f0 = (4 * e) % dp;
      f32x4 v;
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = f0 + u < d ? sx[r * d + f0 + u] : 0.f;
      dst[e] = v;
    }
  }
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= nct) return;
  const float sg = knn_scale(scal);
  const int l = threadIdx.x & 63;
  const int h = l >> 5;
  const int lr = (threadIdx.x >> 6) * 32 + (l & 31);  // row within the block
  const bool valid = lr < rows;
  const float* xc = sx + lr * d;
  float cn = 0.f;
  if (valid)
    for (int f = 0; f < d; ++f) {
      const float y = sg * xc[f];
      cn = fmaf(y, y, cn);
    }
  for (int s = 0; s < KS16; ++s) {
    f16x8 hv, lv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = 16 * s + 8 * h + j;
      float v;
      if (valid)
        v = (f < d) ? -2.f * sg * xc[f] : ((f == d) ? cn : 0.f);
      else
        v = (f == d) ? kPadNorm16 : 0.f;
      _Float16 a, b;
      split_f16(v, a, b);
      hv[j] = a;
      lv[j] = b;
    }
    *reinterpret_cast<f16x8*>(apack + (((t * KS16 + s) * nh) * 64 + l) * 8) = hv;
    if (nh == 2) *reinterpret_cast<f16x8*>(apack + (((t * KS16 + s) * 2 + 1) * 64 + l) * 8) = lv;
  }
}

// ---------------------------------------------------------------------------------------
// 3. refine + certify
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool lex_less_f(float a, int ai, float b, int bi) {
  return a < b || (a == b && ai < bi);
}

// exact_d2 with b a padded candidate row (16-B aligned, zeros past d, length a multiple of 32):
// the same operations in the same order, b read as dwordx4.
__device__ __forceinline__ double exact_d2_pad(const float* __restrict__ a,
                                               const float* __restrict__ b, int d) {
  constexpr int kCh = 32;
  double s = 0.0;
  for (int f0 = 0; f0 < d; f0 += kCh) {
    float av[kCh];
    f32x4 bv[kCh / 4];
#pragma unroll
    for (int u = 0; u < kCh / 4; ++u) bv[u] = reinterpret_cast<const f32x4*>(b + f0)[u];
#pragma unroll
    for (int u = 0; u < kCh; ++u) av[u] = a[min(f0 + u, d - 1)];
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      if (f0 + u < d) {  // uniform condition
        const double t = __dsub_rn((double)av[u], (double)bv[u >> 2][u & 3]);
        s = __dadd_rn(s, __dmul_rn(t, t));
      }
    }
  }
  return s;
}

// exact_d2_pad with the first 32 coordinates of a already in registers (qa[u] = a[min(u, d - 1)]):
// the same operations in the same order.
__device__ __forceinline__ double exact_d2_pad_pre(const float (&qa)[32],
                                                   const float* __restrict__ a,
                                                   const float* __restrict__ b, int d) {
  constexpr int kCh = 32;
  double s = 0.0;
  for (int f0 = 0; f0 < d; f0 += kCh) {
    float av[kCh];
    f32x4 bv[kCh / 4];
#pragma unroll
    for (int u = 0; u < kCh / 4; ++u) bv[u] = reinterpret_cast<const f32x4*>(b + f0)[u];
    if (f0 == 0) {
#pragma unroll
      for (int u = 0; u < kCh; ++u) av[u] = qa[u];
    } else {
#pragma unroll
      for (int u = 0; u < kCh; ++u) av[u] = a[min(f0 + u, d - 1)];
    }
#pragma unroll
    for (int u = 0; u < kCh; ++u) {
      if (f0 + u < d) {  // uniform condition
        const double t = __dsub_rn((double)av[u], (double)bv[u >> 2][u & 3]);
        s = __dadd_rn(s, __dmul_rn(t, t));
      }
    }
  }
  return s;
}

// Lane l's value from lane l ^ M: DPP quad permutes for M = 1, 2 (a VALU move), ds_swizzle's
// xor mode for M = 4 .. 16 (no address operand), ds_bpermute (__shfl_xor) for M = 32.
template <int M>
__device__ __forceinline__ int xor_lane(int v) {
  if constexpr (M == 1)
    return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);  // quad_perm [1, 0, 3, 2]
  else if constexpr (M == 2)
    return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);  // quad_perm [2, 3, 0, 1]
  else if constexpr (M < 32)
    return __builtin_amdgcn_ds_swizzle(v, 0x1F | (M << 10));  // and 31, or 0, xor M
  else
    return __shfl_xor(v, M, kWave);
}
template <int M>
__device__ __forceinline__ double xor_lane(double x) {
  const int2 v = __builtin_bit_cast(int2, x);
  return __builtin_bit_cast(double, make_int2(xor_lane<M>(v.x), xor_lane<M>(v.y)));
}

// One compare-exchange stage of the ascending bitonic sort of 64 (d, i) pairs across the wave.
template <int SIZE, int STRIDE>
__device__ __forceinline__ void bitonic_stage(double& dd, int& di, int l) {
  const double od = xor_lane<STRIDE>(dd);
  const int oi = xor_lane<STRIDE>(di);
  const bool up = (l & SIZE) == 0;
  const bool lower = (l & STRIDE) == 0;
  const bool other_less = lex_less(od, oi, dd, di);
  // lower lane keeps the min if ascending block, max otherwise
  const bool take = (lower == up) ? other_less : !other_less && !(od == dd && oi == di);
  if (take) {
    dd = od;
    di = oi;
  }
  if constexpr (STRIDE > 1) bitonic_stage<SIZE, STRIDE / 2>(dd, di, l);
}
template <int SIZE = 2>
__device__ __forceinline__ void bitonic_sort64(double& dd, int& di, int l) {
  bitonic_stage<SIZE, SIZE / 2>(dd, di, l);
  if constexpr (SIZE < 64) bitonic_sort64<SIZE * 2>(dd, di, l);
}

template <int LIST, int MAXP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void refine_kernel(
    const float* __restrict__ cpad, int dp, int64_t nc, const float* __restrict__ query,
    int64_t nq, int d, int kp1, int M, int list_len, const float* __restrict__ lists_v,
    const int* __restrict__ lists_i, const unsigned* __restrict__ cmax_bits, int e_terms,
    double* __restrict__ Dout,
    int64_t* __restrict__ I64, int32_t* __restrict__ I32, int* __restrict__ flag_count,
    int* __restrict__ flag_list, double* __restrict__ flag_bound, int rank_merge) {
  __shared__ int sel[4][64];
  __shared__ float selv[4][64];  // rank merge: approximate value of sel[r]
  constexpr int kRM = MAXP <= 4 ? MAXP : 1;  // rank merge for M <= 256 entries
  __shared__ float2 sent[4][64 * kRM];        // rank merge: the query's entries (value, index bits)
  if (MAXP > 4) rank_merge = 0;
  // wave-uniform in an SGPR: the query row and the lists' addresses are then scalar, and the
  // query's coordinates come through scalar loads instead of 64-lane broadcast vector loads
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  // XCD-aware block order: workgroups are dealt round-robin over the 8 XCDs, so block b runs on
  // XCD b % 8; each XCD gets one contiguous range of query blocks.  Neighbouring queries' rows of
  // the transposed index table (I32[l][q], 4 bytes per query) then meet in one L2 and leave it
  // as whole lines instead of 16-byte pieces from 8 different L2s.
  const int64_t nb = gridDim.x, bx = blockIdx.x;
  const int64_t xcd = bx & 7, per = nb >> 3, rem = nb & 7;
  const int64_t qb = xcd * per + min(xcd, rem) + (bx >> 3);
  const int64_t q = qb * 4 + w;
  if (q >= nq || skip_screen(cmax_bits)) return;
  // The query row first: |q|^2 and the exact distances' first 32 coordinates are then loaded
  // beside the lists instead of after the merge (the wave fences below keep memory operations
  // from moving across them)
  const float* xq = query + q * d;
  float qa[32];
#pragma unroll
  for (int u = 0; u < 32; ++u) qa[u] = xq[min(u, d - 1)];
  double qn2 = 0.0;
  for (int f = l; f < d; f += 64) qn2 += (double)xq[f] * (double)xq[f];
  // Candidate entries of this query: 2*split ascending partial lists of list_len each, the last
  // slot of each carrying that lane's prune bound (select16_kernel).
  const float* lv = lists_v + q * M;
  const int* lix = lists_i + q * M;
  const int nval = M;

  // Bound part 1: min over partial lists of their last slot (their lanes' final bounds).
  float bnd = INFINITY;
  for (int p = l; p < M / list_len; p += 64) bnd = fminf(bnd, lv[p * list_len + list_len - 1]);

  float ev[MAXP];
  int ei[MAXP];
#pragma unroll
  for (int p = 0; p < MAXP; ++p) {
    const int e = p * 64 + l;
    float v = INFINITY;
    int ix = INT_MAX;
    if (e < nval) {
      // both loads issued before either is tested (a value load behind the index test would
      // wait out a second memory round trip)
      const int ii = __builtin_nontemporal_load(lix + e);
      const float vv = __builtin_nontemporal_load(lv + e);
      const bool ok = ii >= 0 && ii < nc;
      v = ok ? vv : INFINITY;
      ix = ok ? ii : INT_MAX;
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
    if (rank_merge == 2) {
      // Each of the 2 split partial lists is ascending in value: an entry's rank is, per list,
      // a binary search for the entries of smaller value plus the (rare) equal-value entries of
      // smaller index -- O(lists x log LIST16) LDS reads per entry instead of all M.
      const int nl = mtot / list_len;
      const float2* se = sent[w];
      // unrolled: the lists' binary searches are independent LDS read chains
#pragma unroll 4
      for (int s = 0; s < nl; ++s) {
        const float2* L = se + s * list_len;
#pragma unroll
        for (int p = 0; p < MAXP; ++p) {
          int k = 0;
#pragma unroll
          for (int step = 32; step >= 1; step >>= 1)
            if (k + step <= list_len && L[k + step - 1].x < ev[p]) k += step;
          int c = k;
          while (ei[p] != INT_MAX && k < list_len && L[k].x == ev[p]) {
            c += __float_as_int(L[k].y) < ei[p] ? 1 : 0;
            ++k;
          }
          rk[p] += c;
        }
      }
    } else {
#pragma nounroll
      for (int e = 0; e < mtot; ++e) {
        const float2 o = sent[w][e];
        const float ov = o.x;
        const int oi = __float_as_int(o.y);
#pragma unroll
        for (int p = 0; p < MAXP; ++p) rk[p] += lex_less_f(ov, oi, ev[p], ei[p]) ? 1 : 0;
      }
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
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) qn2 += __shfl_xor(qn2, m, kWave);
  const double cmax = (double)__uint_as_float(*cmax_bits);
  // e_terms * 2^-24 * (C^2 + 2 C |q|) bounds the selection's error (make_plan), C = max
  // candidate norm.
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
      dd = exact_d2_pad_pre(qa, xq, cpad + (int64_t)c * dp, d);
      di = c;
    }
  }
  // Bitonic sort of 64 (dd, di) pairs across the wave, ascending (the same network as the
  // round-5 __shfl_xor loop; the partner exchanges by DPP / ds_swizzle where the stride allows)
  bitonic_sort64(dd, di, l);
  // Certification: every candidate outside the exactly evaluated set has exact
  // d^2 >= bnd + |q|^2 - E.
  const double ek = __shfl(dd, kp1 - 1, kWave);
  const int eki = __shfl(di, kp1 - 1, kWave);
  bool ok = eki != INT_MAX;
  if (bnd < 1e29f) ok = ok && (ek < ((double)bnd + qn2) - E);
  if (l < kp1) {
    Dout[q * kp1 + l] = sqrt_rn(dd);
    if (I64) I64[q * kp1 + l] = di;
    if (I32) I32[(int64_t)l * nq + q] = di;  // transposed [kp1][nq]
  }
  if (!ok && l == 0) {
    const int slot = atomicAdd(flag_count, 1);
    flag_list[slot] = (int)q;
    // the (k+1)-th smallest exact d^2 evaluated here bounds the answer's (exact stage)
    flag_bound[slot] = eki != INT_MAX ? ek : INFINITY;
  }
}

// ---------------------------------------------------------------------------------------
// host-side plan + dispatch
// ---------------------------------------------------------------------------------------
struct Plan {
  int d, kp1, LIST, split, maxp;
  int dp;         // padded candidate row (floats, multiple of 32) for refine's gathers
  int KS16;       // k-steps of 16: ceil((d + 1) / 16) <= 4
  int nh;         // candidate halves in the fragments: 1 (hi, default) or 2 (hi + lo)
  int e_terms;    // selection error bound multiplier (refine certification)
  int keep;       // per-half entries behind the union prune bound
  int LIST16;     // per-half select list length
  int M;          // refine input entries per query: 2*split*LIST16
  int64_t nc, nq, nct, nqt, tiles_per_split;
  bool exhaustive;  // no f16 screen: every query scanned exactly (knn_exact.hip block select)
  size_t off_apack, off_scalars, off_lv, off_li, off_flag, off_fbound, off_part, off_cpad, off_seed;
  size_t off_candT, off_wbuf, total;
};

// The f16 screen (select + refine) covers d <= kScreenMaxD (4 k-steps of 16 with the norm
// column) and k + 1 <= kScreenMaxKp1 (two half lists of <= 40 behind the union bound, refine's
// 64 ranked entries); every other shape takes the exhaustive plan.
constexpr int kScreenMaxD = 63;
constexpr int kScreenMaxKp1 = 60;

// Exhaustive plan: validation scalars, the transposed candidates and (kp1 beyond the LDS
// capacity) the block-select buffers.
static int make_exhaustive_plan(Plan* P) {
  size_t off = 0;
  P->exhaustive = true;
  P->split = 0;
  P->LIST16 = wide_cap(P->kp1);
  P->KS16 = 0;
  P->nh = 0;
  P->off_scalars = off;
  off = align_up(off + 32, 256);
  P->off_candT = off;
  off = align_up(off + (size_t)P->nc * P->d * sizeof(float), 256);
  P->off_wbuf = off;
  off = align_up(off + wide_buffer_bytes(P->nq, 1, P->kp1), 256);
  P->total = off;
  return 0;
}

// 22 = keep + 4 at k + 1 = 31; keep + 2 (20 there) makes the select 3 % faster but sends 43
// instead of 1 of 200k queries to the exhaustive stage, slower overall (round 5,
// profiles/r5/knn/list_slack_ab.txt)
static const int kListChoices[] = {8, 16, 20, 22, 24, 32, 40};

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
  P->d = d;
  P->kp1 = kp1;
  P->nc = nc;
  P->nq = nq;
  P->exhaustive = false;
  if (d > kScreenMaxD || kp1 > kScreenMaxKp1) return make_exhaustive_plan(P);
  P->KS16 = (d + 1 + 15) / 16;
  // f16 lists: each half-lane keeps LIST16 entries and prunes against the union bound
  // (flush_groups, keep = ceil(kp1/2) + 2 per half: 2 keep >= kp1 + 3).  A half holding more
  // than LIST16 of the query's nearest candidates only costs certification (exact path).
  P->keep = (kp1 + 1) / 2 + 2;
  P->LIST16 = 40;
  for (int v : kListChoices)
    if (v >= P->keep + 4) {
      P->LIST16 = v;
      break;
    }
  // Candidate halves.  The hi-only band E ~ 3 * 2^-11 C^2 must stay small against the
  // (k+1)-th neighbour distance, ~C^2 (kp1 / nc)^(2/d) for nc points spread over the radius-C
  // ball: at C3 / C4 / C5 the ratio is ~0.003, for low-dimensional dense data (GridWorld,
  // MountainCar, d = 2) it exceeds 1 and nearly every query would go to the exhaustive path.
  // Split candidates (E ~32x smaller) cover those.  MEPOL_KNN_NH=1|2 forces either.
  {
    const double band = 3.0 / 2048.0 * std::pow((double)nc / kp1, 2.0 / d);
    P->nh = band > 0.03 ? 2 : 1;
    const char* e = getenv("MEPOL_KNN_NH");
    if (e && (e[0] == '1' || e[0] == '2')) P->nh = e[0] - '0';
    // split-candidate instances that stay below the 256-VGPR cap
    const bool fits2 = (P->KS16 <= 3 && P->LIST16 <= (P->KS16 == 3 ? 32 : 40)) ||
                       (P->KS16 == 4 && P->LIST16 <= 32);
    if (!fits2) P->nh = 1;
  }
  // Selection error bound E = e_terms * 2^-24 * (C^2 + 2 C |q|), unscaled, C = max candidate
  // norm.  Candidate-hi: the f16 rounding of -2 sigma c and of |sigma c|^2 (2^-11 = 2^13 * 2^-24
  // relative each: 2^-11 (2 |c||q| + |c|^2)), the query split (2^-22), the 2 K products per
  // output summed in f32 (<= 2K roundings) and |c|^2 in f32 (d roundings), these small terms
  // x2, and 64 for the f16 subnormal range.  Split candidates: 3 K products summed in f32,
  // operand splitting 3 * 2^-22 = 12 * 2^-24, |c|^2 in f32 (d), x2.
  P->e_terms = P->nh == 1 ? 8192 + 64 + 2 * (2 * 16 * P->KS16 + 16 + d)
                          : 2 * (3 * 16 * P->KS16 + 16 + d);
  // Candidate-hi plans with <= 3 k-steps (d <= 47) drop the query's lo half too
  // (select16_kernel: kQueryLo): its f16 rounding, 2^-11 2 |c||q| (+64 for subnormals), joins
  // the bound.  Measured C3 7.0 -> 5.7 ms, d = 47 9.9 -> 8.0 ms with no added fallbacks; at d = 63,
  // k+1 = 51 (C5) the wider band sent 1633 of 500k queries to the exhaustive path (8 with it),
  // so 4-step plans keep it (profiles/r4/knn/qlo_ab_probe.log).
  if (P->nh == 1 && P->KS16 <= 3) P->e_terms += 8192 + 64;
  // the selection's error band (~0.1 at C3) holds a few more candidates around the (k+1)-th
  // than kp1 + 4: refine ranks the approximate top 64 and evaluates those inside the band
  P->LIST = kRefineList;
  P->nct = (nc + 31) / 32;
  P->nqt = (nq + 31) / 32;
  int split = split_hint;
  if (split <= 0) {
    // About 1600 query-tile waves (half of the 3072 wave slots at 3 waves per SIMD), tiles
    // >= 16 per split.  Every (query, split) pays the list warm-up (the prune bound starts at
    // +inf, or at a finished range's bound) and refine ranks 2 split LIST16 entries per query,
    // so fewer, longer ranges win even below a full chip: 25k queries x 200k (the C3 shard at
    // 8 ranks) take 1.25 ms at split 2, 1.30 at 3, 1.54 at 4, 1.94 at 8; 200k queries 5.27 ms at
    // 2, 5.62 at 3, 5.97 at 4 (round 5, profiles/r5/knn/splits.txt).  The lists keep >= 2
    // ranges (one range of half lists certifies too few queries).
    const int64_t target = 1600;
    split = (int)std::min<int64_t>(kMaxSplit, std::max<int64_t>(1, (target + P->nqt / 2) /
                                                                      std::max<int64_t>(P->nqt, 1)));
    split = std::max(split, 2);
    // refine's rank merge takes <= 256 entries per query (2 split LIST16)
    split = std::min(split, std::max(2, 256 / (2 * P->LIST16)));
    while (split > 1 && P->nct / split < 16) --split;
  }
  split = std::max(1, std::min(split, kMaxSplit));
  P->split = split;
  P->tiles_per_split = (P->nct + split - 1) / split;
  P->M = 2 * split * P->LIST16;
  P->maxp = (P->M + 63) / 64;
  if (P->maxp > 32) {
    set_error("mepol_knn: refine capacity %d entries per query exceeds 2048", P->M);
    return kErrUnsupported;
  }
  size_t off = 0;
  P->off_apack = off;
  off = align_up(off + (size_t)P->nct * 64 * P->KS16 * 16 * sizeof(_Float16), 256);  // nh <= 2
  P->off_scalars = off;  // [0] max |c| bits, [1] fallback count, [2] max |q| bits, [4..5] invalid rows
  off = align_up(off + 32, 256);
  const size_t nl = (size_t)std::max<int64_t>(nq, 1) * P->M;
  P->off_lv = off;
  off = align_up(off + nl * sizeof(float), 256);
  P->off_li = off;
  off = align_up(off + nl * sizeof(int), 256);
  P->off_flag = off;
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(int), 256);
  P->off_fbound = off;  // refine's bound per queued query (exact stage)
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(double), 256);
  P->off_part = off;  // exact fallback: kExactGrid partial lists of <= 64 (f64, int32)
  off = align_up(off + (size_t)kExactGrid * 64 * (sizeof(double) + sizeof(int)), 256);
  P->dp = (d + 31) / 32 * 32;
  P->off_cpad = off;
  off = align_up(off + (size_t)nc * P->dp * sizeof(float), 256);
  P->off_seed = off;  // per-query prune-bound seeds (select16_kernel)
  off = align_up(off + (size_t)std::max<int64_t>(nq, 1) * sizeof(int), 256);
  P->off_candT = P->off_wbuf = 0;
  P->total = off;
  return 0;
}

// Prune-bound seeds of the selection: 2 (default) = the probe sample's bound (probe16_kernel)
// and the bounds finished candidate ranges publish; MEPOL_KNN_SEED=1: the published bounds only
// (round 5); 0: every candidate range starts its prune bound at +inf.  The certified output is
// the same bits either way (tests/test_gpu_knn.py::test_knn_seed_invariance); only the partial
// lists, and so the count of queries sent to the exhaustive stage, differ.
static int select_seed() {
  const char* e = getenv("MEPOL_KNN_SEED");
  return (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : 2;
}

// refine_kernel's merge of the partial lists: per-list binary-search ranks (2); the kernel
// keeps the full-count ranks (1) and argmin rounds (0) for MAXP > 4 plans.
constexpr int kRankMerge = 2;

static void launch_refine(const Plan& P, const float* cpad, const float* query, const float* lv,
                          const int* li, const unsigned* cmax, double* D, int64_t* I64,
                          int32_t* I32, int* fc, int* fl, double* fb, hipStream_t st) {
  dim3 g((unsigned)((P.nq + 3) / 4));
  // MAXP = ceil(M / 64) <= 32
#define MEPOL_REFINE(MP)                                                                          \
  hipLaunchKernelGGL((refine_kernel<kRefineList, MP>), g, dim3(256), 0, st, cpad, P.dp, P.nc,     \
                     query, P.nq, P.d, P.kp1, P.M, P.LIST16, lv, li, cmax, P.e_terms, D, I64,     \
                     I32, fc, fl, fb, kRankMerge)
  if (P.maxp <= 2)
    MEPOL_REFINE(2);
  else if (P.maxp <= 4)
    MEPOL_REFINE(4);
  else if (P.maxp <= 8)
    MEPOL_REFINE(8);
  else if (P.maxp <= 16)
    MEPOL_REFINE(16);
  else
    MEPOL_REFINE(32);
#undef MEPOL_REFINE
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
  if (ks) *ks = P.KS16 * 10 + P.nh;  // k-steps of 16, candidate halves
  if (list) *list = P.LIST16;
  if (split) *split = P.split;
  return 0;
}

// invalid_out == nullptr: validate on the host (one stream synchronisation after the norms pass,
// like the reference's blocking kneighbors).  Otherwise the two counts go to invalid_out on the
// device and the call never blocks (mepol_knn_deferred).
static int knn_impl(const float* cand, int64_t n_cand, const float* query, int64_t n_query, int d,
                    int kp1, int split_hint, double* dist_out, int64_t* idx_out,
                    int32_t* idx32_out, int32_t* n_fallback_out, int32_t* invalid_out,
                    void* workspace, size_t workspace_bytes, void* stream) {
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
  unsigned* cmax = (unsigned*)(ws + P.off_scalars);
  int* fcount = n_fallback_out ? (int*)n_fallback_out : (int*)(ws + P.off_scalars + 4);
  MEPOL_HIP(hipMemsetAsync(ws + P.off_scalars, 0, 32, st));
  if (n_fallback_out) MEPOL_HIP(hipMemsetAsync(n_fallback_out, 0, sizeof(int32_t), st));
  const bool self_query = query == cand && P.nq == P.nc;
  ExactArgs ea{cand,     nullptr,  P.nc,    query,  P.nq,    P.d,     P.kp1,   fcount,
               nullptr,  cmax,     0,       dist_out, idx_out, idx32_out, nullptr, nullptr,
               nullptr,  nullptr};
  // 0. validation (+ the transposed candidates of an exhaustive plan)
  if (P.exhaustive) {
    ea.candT = (float*)(ws + P.off_candT);
    launch_transpose_validate(cand, P.nc, P.d, (float*)ea.candT, cmax + 4, st);
    if (!self_query) launch_transpose_validate(query, P.nq, P.d, nullptr, cmax + 4, st);
  } else {
    // scal[0] = max candidate norm (refine's C), scal[2] = max query norm (f16 scale)
    const size_t stage_lds = (size_t)kStageRows * P.d * sizeof(float);  // <= 32 KB (d <= 63)
    auto norms_grid = [](int64_t rows) {
      return dim3((unsigned)std::min<int64_t>(kNormsBlocks, (rows + kStageRows - 1) / kStageRows));
    };
    hipLaunchKernelGGL(norms_kernel, norms_grid(P.nc), dim3(kNormsThreads), stage_lds, st, cand,
                       P.nc, P.d, cmax, cmax + 4, self_query ? cmax + 2 : nullptr);
    if (!self_query)
      hipLaunchKernelGGL(norms_kernel, norms_grid(P.nq), dim3(kNormsThreads), stage_lds, st,
                         query, P.nq, P.d, cmax + 2, cmax + 4, nullptr);
  }
  MEPOL_CHECK_LAUNCH();
  if (invalid_out) {
    MEPOL_HIP(hipMemcpyAsync(invalid_out, cmax + 4, 2 * sizeof(int32_t), hipMemcpyDeviceToDevice,
                             st));
  } else {
    // sklearn rejects non-finite input (ValueError from check_array): validate before the scan.
    // Rows whose f32 squared norm overflows (bad[1]) are valid input: the f16 screen cannot
    // scale them, so every query goes to the exhaustive f64 stage (ExactArgs).
    unsigned bad[2] = {0, 0};
    MEPOL_HIP(hipMemcpyAsync(bad, cmax + 4, sizeof(bad), hipMemcpyDeviceToHost, st));
    MEPOL_HIP(hipStreamSynchronize(st));
    if (bad[0]) {
      set_error("mepol_knn: Input contains NaN or infinity (%u rows)", bad[0]);
      return kErrBadArg;
    }
    if (bad[1] && wide_buffer_bytes(P.nq, 1, P.kp1) == 0) {
      // Every query goes to the exhaustive stage: take its fast form over the whole grid (the
      // transposed candidates, in the padded-row area the screen would have used: nc * dp >=
      // nc * d floats) instead of the queued-query form the screen's fallback uses.
      ea.candT = (float*)(ws + P.off_cpad);
      launch_transpose_validate(cand, P.nc, P.d, (float*)ea.candT, nullptr, st);
      ea.all = 1;
      ea.scal = nullptr;
      ea.wbuf_d = nullptr;
      ea.wbuf_i = nullptr;
      if (n_fallback_out)
        MEPOL_HIP(hipMemsetD32Async((hipDeviceptr_t)n_fallback_out, (int)P.nq, 1, st));
      launch_exact_stage(ea, st);
      MEPOL_CHECK_LAUNCH();
      return 0;
    }
  }
  if (P.exhaustive) {
    ea.all = 1;
    ea.wbuf_d = (double*)(ws + P.off_wbuf);
    ea.wbuf_i = (int*)(ws + P.off_wbuf +
                       (size_t)wide_grid(P.nq, 1, P.kp1) * wide_cap(P.kp1) * sizeof(double));
    if (n_fallback_out)
      MEPOL_HIP(hipMemsetD32Async((hipDeviceptr_t)n_fallback_out, (int)P.nq, 1, st));
    launch_exact_stage(ea, st);
    MEPOL_CHECK_LAUNCH();
    return 0;
  }
  _Float16* ap16 = (_Float16*)(ws + P.off_apack);
  float* lv = (float*)(ws + P.off_lv);
  int* li = (int*)(ws + P.off_li);
  float* cpad = (float*)(ws + P.off_cpad);
  const size_t stage_lds = (size_t)kStageRows * P.d * sizeof(float);
  hipLaunchKernelGGL(pack16_kernel, dim3((unsigned)((P.nct + 3) / 4)), dim3(256), stage_lds, st,
                     cand, P.nc, P.d, P.KS16, P.nh, P.nct, ap16, cmax, cpad, P.dp);
  MEPOL_CHECK_LAUNCH();
  {
    int* seed = nullptr;
    int seeding = select_seed();
    // The probe seed leaves ~kProbeKth * nc / (32 np) candidates below it (the smaller of the two
    // lanes' kProbeKth-th tile minima over np sampled tiles); it pays only where that is far
    // above k + 1.  Split-candidate plans (low-dimensional, duplicate-heavy data: GridWorld,
    // MountainCar) keep the published bounds only: exact ties at a tight seed would cost
    // certification (measured: C2S k-NN 1.5 -> 10.9 ms with the probe).
    if (seeding == 2) {
      const double np = (double)std::min<int64_t>(kProbeTiles, P.nct);
      const double below = kProbeKth * (double)P.nc / (32.0 * np);
      if (P.nh != 1 || below < 4.0 * P.kp1) seeding = 1;
    }
    if (seeding == 2 || (seeding == 1 && P.split > 1)) {
      seed = (int*)(ws + P.off_seed);
      // the probe kernel writes every query's seed; without it ranges start from +inf
      if (seeding == 1)
        MEPOL_HIP(hipMemsetD32Async((hipDeviceptr_t)seed, kSeedNone, (size_t)P.nq, st));
    }
    const SelectArgs sa{ap16,   query,    P.nq, P.d,   P.nct, P.split, P.tiles_per_split,
                        P.keep, P.LIST16, P.nh, P.nqt, cmax,  lv,      li,
                        seed,   seeding == 2};
    switch (P.KS16) {
      case 1: launch_select<1>(sa, st); break;
      case 2: launch_select<2>(sa, st); break;
      case 3: launch_select<3>(sa, st); break;
      default: launch_select<4>(sa, st); break;
    }
  }
  MEPOL_CHECK_LAUNCH();
  int* flist = (int*)(ws + P.off_flag);
  double* fbound = (double*)(ws + P.off_fbound);
  launch_refine(P, cpad, query, lv, li, cmax, dist_out, idx_out, idx32_out, fcount, flist, fbound,
                st);
  MEPOL_CHECK_LAUNCH();
  // 4. queued queries (or all of them, scal[5]) by the exhaustive stage
  ea.flag_list = flist;
  ea.flag_bound = fbound;
  ea.part_d = (double*)(ws + P.off_part);
  ea.part_i = (int*)(ws + P.off_part + (size_t)kExactGrid * 64 * sizeof(double));
  launch_exact_stage(ea, st);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_knn(const float* cand, int64_t n_cand, const float* query, int64_t n_query,
                         int d, int kp1, int split_hint, double* dist_out, int64_t* idx_out,
                         int32_t* idx32_out, int32_t* n_fallback_out, void* workspace,
                         size_t workspace_bytes, void* stream) {
  return knn_impl(cand, n_cand, query, n_query, d, kp1, split_hint, dist_out, idx_out, idx32_out,
                  n_fallback_out, nullptr, workspace, workspace_bytes, stream);
}

extern "C" int mepol_knn_deferred(const float* cand, int64_t n_cand, const float* query,
                                  int64_t n_query, int d, int kp1, int split_hint,
                                  double* dist_out, int64_t* idx_out, int32_t* idx32_out,
                                  int32_t* n_fallback_out, int32_t* invalid_out, void* workspace,
                                  size_t workspace_bytes, void* stream) {
  if (!invalid_out) {
    set_error("mepol_knn_deferred: null invalid_out");
    return kErrBadArg;
  }
  return knn_impl(cand, n_cand, query, n_query, d, kp1, split_hint, dist_out, idx_out, idx32_out,
                  n_fallback_out, invalid_out, workspace, workspace_bytes, stream);
}

// Exhaustive exact k-NN for every query (no f16 screen, no validation, no workspace): the
// reference semantics at the cost of a full f64 scan over row-major candidates; an independent
// check of mepol_knn.  kp1 <= 3072 (its block-select lists live in LDS); scratch_idx is unused
// (kept for the ABI).
extern "C" int mepol_knn_exact(const float* cand, int64_t n_cand, const float* query,
                               int64_t n_query, int d, int kp1, double* dist_out, int64_t* idx_out,
                               int32_t* idx32_out, int32_t* scratch_idx, void* stream) {
  (void)scratch_idx;
  if (n_cand <= 0 || n_query < 0 || d <= 0 || kp1 <= 0 || kp1 > n_cand || !cand || !query ||
      !dist_out) {
    set_error("mepol_knn_exact: bad arguments (needs 0 < k+1 <= n_cand)");
    return kErrBadArg;
  }
  if (n_cand > INT_MAX - 64) {
    set_error("mepol_knn_exact: n_cand=%lld exceeds int32 indexing", (long long)n_cand);
    return kErrUnsupported;
  }
  if (wide_buffer_bytes(n_query, 1, kp1) > 0) {
    set_error("mepol_knn_exact: k+1=%d beyond its LDS lists (mepol_knn takes any k+1)", kp1);
    return kErrUnsupported;
  }
  if (n_query == 0) return 0;
  const ExactArgs ea{cand, nullptr, n_cand, query, n_query, d, kp1, nullptr, nullptr, nullptr, 1,
                     dist_out, idx_out, idx32_out, nullptr, nullptr, nullptr, nullptr};
  launch_exact_stage(ea, (hipStream_t)stream);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
