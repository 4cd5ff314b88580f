// The exhaustive stage of the k-NN (step 4 of knn.hip's pipeline): exact f64 distances of a
// query to every candidate, in feature order with no contraction (the reference's sklearn
// kd_tree arithmetic, src/algorithms/mepol.py:190-192), top-kp1 by (distance, index).
//
// Two forms:
//   * register lists (kp1 <= 64): each thread keeps a sorted list of its candidates, kp1 rounds
//     of block argmin merge them.  With few queued queries, a query's candidates are cut into
//     chunks spread over the grid (partial lists + exact_merge_kernel).
//   * block select (any kp1 <= nc, any d): the block's threads append every candidate below
//     the query's running kp1-th (distance, index) to a shared buffer; when the buffer fills, a
//     bitonic sort keeps the first kp1 and tightens the threshold.  The buffer is in LDS up to
//     kWideLdsCap entries and in a caller-owned global workspace beyond.  Candidates are read
//     from a transposed copy [d][nc] (one coalesced load per feature and 64 candidates) when the
//     plan made one, else row-major.
// This form answers every query of the plans the f16 screen does not cover (knn.hip make_plan:
// d > 63, kp1 > 60) and the queued queries of those that it does.
#include "knn_common.hpp"

namespace mepol {
namespace knn {

// Queries of the stage (ExactArgs): returns the count, 0 for a rejected input.
__device__ __forceinline__ int stage_count(const ExactArgs& a) {
  if (a.scal && a.scal[4]) return 0;
  return (a.all || (a.scal && a.scal[5])) ? (int)a.nq : *a.flag_count;
}
__device__ __forceinline__ int64_t stage_query(const ExactArgs& a, int fi) {
  return (a.all || (a.scal && a.scal[5])) ? (int64_t)fi : (int64_t)a.flag_list[fi];
}
// A screened plan whose input the screen could not scale reports every query as answered by
// this stage (the count the caller reads as n_fallback).  One thread of the stage's first kernel.
__device__ __forceinline__ void stage_report(const ExactArgs& a) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && !a.all && a.scal && !a.scal[4] && a.scal[5])
    *a.flag_count = (int)a.nq;
}

// ---------------------------------------------------------------------------------------
// register lists (kp1 <= 64)
// ---------------------------------------------------------------------------------------
// Exhaustive f64 top-kp1 of query xq over candidates [c0, c1), lexicographic (dist, idx):
// per-thread sorted lists, then kp1 rounds of block argmin; round r's winner goes to
// emit(r, d, i) on thread 0 (i = INT_MAX, d = inf when the range holds fewer than kp1).
// ub: only candidates with d^2 <= ub can be among the first kp1 (refine's bound for a queued
// query, +inf otherwise): the others are never inserted.
template <int LIST, typename Emit>
__device__ __forceinline__ void exact_scan(const float* __restrict__ cand, int64_t c0, int64_t c1,
                                           const float* __restrict__ xq, int d, int kp1,
                                           double ub, double* red_d, int* red_i, Emit emit) {
  const int tid = threadIdx.x;
  const int l = tid & 63, w = tid >> 6;
  double ld[LIST];
  int li[LIST];
#pragma unroll
  for (int j = 0; j < LIST; ++j) {
    ld[j] = INFINITY;
    li[j] = INT_MAX;
  }
#pragma nounroll
  for (int64_t c = c0 + tid; c < c1; c += blockDim.x) {
    const double x = exact_d2(xq, cand + c * d, d);
    const int xi = (int)c;
    if (x <= ub && lex_less(x, xi, ld[LIST - 1], li[LIST - 1])) {
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
    if (li[0] == bi && bi != INT_MAX) {
#pragma unroll
      for (int j = 0; j < LIST - 1; ++j) {
        ld[j] = ld[j + 1];
        li[j] = li[j + 1];
      }
      ld[LIST - 1] = INFINITY;
      li[LIST - 1] = INT_MAX;
    }
    if (tid == 0) emit(r, bd, bi);
    if (bi == INT_MAX) {  // block-uniform: every list is empty, the rest are +inf too
      if (tid == 0)
        for (int rr = r + 1; rr < kp1; ++rr) emit(rr, (double)INFINITY, INT_MAX);
      break;
    }
  }
}

// With fewer queries than blocks each query's candidates are cut into nchunk = grid / count
// ranges, one block each (partial top-kp1 lists to part_*, merged by exact_merge_kernel): a
// handful of queries then use the whole chip instead of one CU each.  With part_d == nullptr
// or count >= grid, a block answers whole queries.
__host__ __device__ inline int exact_nchunk(int count, int grid) {
  return (count <= 0 || count >= grid) ? 1 : grid / count;
}

// Refine's bound for queued query fi (round 6): its candidates beyond the (k+1)-th exact d^2 that
// refine evaluated cannot be among the first k+1, so the scan inserts almost only the answer
// (C2S, ~600-1300 queued queries on dense d = 2 data: the per-thread list insertions were the
// stage's cost).  The relative slack only admits more candidates; the answer is the same.
__device__ __forceinline__ double stage_bound(const ExactArgs& a, int fi) {
  if (!a.flag_bound || a.all || (a.scal && a.scal[5])) return INFINITY;
  const double b = a.flag_bound[fi];
  return b * (1.0 + 0x1p-40);
}

// bitonic sort and block select of one query (defined with the block-select form below)
__device__ void block_sort(double* bd, int* bi, int n, int P);
constexpr int kExactLdsCap = 2048;  // exact_kernel's block-select buffer: kp1 <= 64, cap - step
template <bool kTransposed>
__device__ void wide_query(const ExactArgs& a, int64_t q, double ub, double* bd, int* bi, int cap,
                           int* s_cnt);

template <int LIST>
__global__ __launch_bounds__(256) void exact_kernel(ExactArgs a) {
  __shared__ double red_d[4];
  __shared__ int red_i[4];
  const int count = stage_count(a);
  stage_report(a);
  const int nchunk = a.part_d ? exact_nchunk(count, (int)gridDim.x) : 1;
  if (nchunk == 1) {
    __shared__ double s_bd[kExactLdsCap];
    __shared__ int s_bi[kExactLdsCap];
    __shared__ int s_cnt;
    for (int fi = blockIdx.x; fi < count; fi += gridDim.x) {
      const int64_t q = stage_query(a, fi);
      const double ub = stage_bound(a, fi);
      if (ub < INFINITY) {  // block-uniform
        // refine's bound leaves ~k+1 candidates: append them to LDS and sort them once instead
        // of per-thread lists and k+1 block argmin rounds (C2S: 500-1300 queued queries)
        wide_query<false>(a, q, ub, s_bd, s_bi, kExactLdsCap, &s_cnt);
        continue;
      }
      exact_scan<LIST>(a.cand, 0, a.nc, a.query + q * a.d, a.d, a.kp1, stage_bound(a, fi), red_d,
                       red_i,
                       [&](int r, double bd, int bi) {
                         a.D[q * a.kp1 + r] = sqrt_rn(bd);
                         if (a.I64) a.I64[q * a.kp1 + r] = bi;
                         if (a.I32) a.I32[(int64_t)r * a.nq + q] = bi;  // transposed [kp1][nq]
                       });
    }
    return;
  }
  const int fi = (int)blockIdx.x / nchunk, ch = (int)blockIdx.x % nchunk;
  if (fi >= count) return;
  const int64_t q = stage_query(a, fi);
  const int64_t c0 = a.nc * ch / nchunk, c1 = a.nc * (ch + 1) / nchunk;
  const int64_t o = ((int64_t)fi * nchunk + ch) * a.kp1;
  exact_scan<LIST>(a.cand, c0, c1, a.query + q * a.d, a.d, a.kp1, stage_bound(a, fi), red_d,
                   red_i,
                   [&](int r, double bd, int bi) {
                     a.part_d[o + r] = bd;
                     a.part_i[o + r] = bi;
                   });
}

// Merge of the nchunk sorted partial lists of one queued query (exact_kernel, chunked form):
// kp1 rounds of block argmin over the list heads; grid = the exact kernel's grid.
__global__ __launch_bounds__(256) void exact_merge_kernel(ExactArgs a, int grid) {
  __shared__ double red_d[4];
  __shared__ int red_i[4];
  __shared__ int red_t[4];
  const int count = stage_count(a);
  const int nchunk = exact_nchunk(count, grid);
  const int fi = blockIdx.x;
  if (nchunk == 1 || fi >= count) return;
  const int kp1 = a.kp1;
  const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
  const int64_t q = stage_query(a, fi);
  const int64_t base = (int64_t)fi * nchunk * kp1;
  if (stage_bound(a, fi) < INFINITY) {  // block-uniform
    // The chunks kept only candidates within refine's bound (a few times k+1 in all): gather
    // the finite entries of the partial lists and sort them once (k+1 rounds of block argmin
    // over 512 list heads took ~58 us for the one queued query of a C3 call).
    __shared__ double s_bd[kExactLdsCap];
    __shared__ int s_bi[kExactLdsCap];
    __shared__ int s_n;
    if (tid == 0) s_n = 0;
    __syncthreads();
    for (int e = tid; e < nchunk * kp1; e += 256) {
      const double x = a.part_d[base + e];
      if (x < INFINITY) {
        const int slot = atomicAdd(&s_n, 1);
        if (slot < kExactLdsCap) {
          s_bd[slot] = x;
          s_bi[slot] = a.part_i[base + e];
        }
      }
    }
    __syncthreads();
    const int n = s_n;
    if (n <= kExactLdsCap) {  // block-uniform; else the argmin rounds below
      int P = 1;
      while (P < n || P < kp1) P <<= 1;
      block_sort(s_bd, s_bi, n, P);  // (distance, index): the same order as the rounds
      for (int r = tid; r < kp1; r += 256) {
        a.D[q * kp1 + r] = sqrt_rn(s_bd[r]);
        if (a.I64) a.I64[q * kp1 + r] = s_bi[r];
        if (a.I32) a.I32[(int64_t)r * a.nq + q] = s_bi[r];  // transposed [kp1][nq]
      }
      return;
    }
  }
  constexpr int kPer = 2;  // lists per thread: nchunk <= grid <= 512
  int pos[kPer] = {0, 0};
  for (int r = 0; r < kp1; ++r) {
    double bd = INFINITY;
    int bi = INT_MAX, bt = -1;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int ch = tid + u * 256;
      if (ch < nchunk && pos[u] < kp1) {
        const double x = a.part_d[base + (int64_t)ch * kp1 + pos[u]];
        const int xi = a.part_i[base + (int64_t)ch * kp1 + pos[u]];
        if (lex_less(x, xi, bd, bi)) {
          bd = x;
          bi = xi;
          bt = u;
        }
      }
    }
    int owner = bt >= 0 ? tid * kPer + bt : INT_MAX;  // which (thread, list) holds the winner
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const double od = __shfl_xor(bd, m, kWave);
      const int oi = __shfl_xor(bi, m, kWave);
      const int ot = __shfl_xor(owner, m, kWave);
      if (lex_less(od, oi, bd, bi) || (od == bd && oi == bi && ot < owner)) {
        bd = od;
        bi = oi;
        owner = ot;
      }
    }
    if (l == 0) {
      red_d[w] = bd;
      red_i[w] = bi;
      red_t[w] = owner;
    }
    __syncthreads();
    bd = red_d[0];
    bi = red_i[0];
    owner = red_t[0];
#pragma unroll
    for (int u = 1; u < 4; ++u)
      if (lex_less(red_d[u], red_i[u], bd, bi) ||
          (red_d[u] == bd && red_i[u] == bi && red_t[u] < owner)) {
        bd = red_d[u];
        bi = red_i[u];
        owner = red_t[u];
      }
    __syncthreads();
    if (owner != INT_MAX && owner / kPer == tid) ++pos[owner % kPer];
    if (tid == 0) {
      a.D[q * kp1 + r] = sqrt_rn(bd);
      if (a.I64) a.I64[q * kp1 + r] = bi;
      if (a.I32) a.I32[(int64_t)r * a.nq + q] = bi;  // transposed [kp1][nq]
    }
  }
}

// ---------------------------------------------------------------------------------------
// block select (any kp1, any d)
// ---------------------------------------------------------------------------------------
constexpr int kWideThreads = 256;
constexpr int kWideUnroll = 4;                            // candidates per thread and step
constexpr int kWideStep = kWideThreads * kWideUnroll;     // candidates per block step
constexpr int kWideLdsCap = 4096;                         // entries kept in LDS (48 KB)
constexpr int kWideGrid = 2048;                           // blocks (all-query plans)
constexpr size_t kWideGlobalBudget = size_t(512) << 20;   // global-buffer bytes at most

int wide_cap(int kp1) {
  int cap = 2048;
  while (cap < kp1 + kWideStep) cap *= 2;
  return cap;
}

int wide_grid(int64_t nq, int all, int kp1) {
  const int cap = wide_cap(kp1);
  int64_t g = all ? std::min<int64_t>(std::max<int64_t>(nq, 1), kWideGrid) : kExactGrid;
  if (cap > kWideLdsCap) {
    const int64_t per = (int64_t)cap * (sizeof(double) + sizeof(int));
    g = std::max<int64_t>(1, std::min<int64_t>(g, (int64_t)(kWideGlobalBudget / per)));
  }
  return (int)g;
}

size_t wide_buffer_bytes(int64_t nq, int all, int kp1) {
  const int cap = wide_cap(kp1);
  if (cap <= kWideLdsCap) return 0;
  return (size_t)wide_grid(nq, all, kp1) * cap * (sizeof(double) + sizeof(int));
}

// Bitonic sort of bd/bi[0, P) ascending by (distance, index), P a power of two; entries
// [n, P) are padding.  Every thread of the block calls it.
__device__ void block_sort(double* bd, int* bi, int n, int P) {
  const int tid = threadIdx.x;
  for (int i = n + tid; i < P; i += kWideThreads) {
    bd[i] = INFINITY;
    bi[i] = INT_MAX;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride >= 1; stride >>= 1) {
      for (int i = tid; i < (P >> 1); i += kWideThreads) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const double dl = bd[lo], dh = bd[hi];
        const int il = bi[lo], ih = bi[hi];
        if (up ? lex_less(dh, ih, dl, il) : lex_less(dl, il, dh, ih)) {
          bd[lo] = dh;
          bi[lo] = ih;
          bd[hi] = dl;
          bi[hi] = il;
        }
      }
      __syncthreads();
    }
  }
}

// Block select of one query: the block appends every candidate below the running kp1-th
// (distance, index) -- from ub on, refine's bound for a queued query, +inf otherwise -- to bd/bi
// (cap entries, LDS or global), compacts to the first kp1 by a bitonic sort when the buffer
// fills, and writes the first kp1.  Every thread of the block calls it.
template <bool kTransposed>
__device__ void wide_query(const ExactArgs& a, int64_t q, double ub, double* bd, int* bi, int cap,
                           int* s_cnt) {
  const int tid = threadIdx.x;
  const int d = a.d, kp1 = a.kp1;
  const int64_t nc = a.nc;
  const float* __restrict__ qrow = a.query + q * d;
  if (tid == 0) *s_cnt = 0;
  __syncthreads();
  double thr_d = ub;  // the running kp1-th (distance, index), block-uniform
  int thr_i = INT_MAX;
  for (int64_t c0 = 0; c0 < nc; c0 += kWideStep) {
    double s[kWideUnroll];
    int64_t cl[kWideUnroll];
#pragma unroll
    for (int u = 0; u < kWideUnroll; ++u) {
      s[u] = 0.0;
      cl[u] = min(c0 + u * kWideThreads + tid, nc - 1);  // clamped: loads stay in bounds
    }
#pragma unroll 2
    for (int f = 0; f < d; ++f) {
      const double qf = (double)qrow[f];
      float x[kWideUnroll];
#pragma unroll
      for (int u = 0; u < kWideUnroll; ++u)
        x[u] = kTransposed ? a.candT[(int64_t)f * nc + cl[u]] : a.cand[cl[u] * d + f];
#pragma unroll
      for (int u = 0; u < kWideUnroll; ++u) {
        const double t = __dsub_rn(qf, (double)x[u]);
        s[u] = __dadd_rn(s[u], __dmul_rn(t, t));
      }
    }
#pragma unroll
    for (int u = 0; u < kWideUnroll; ++u) {
      const int64_t c = c0 + u * kWideThreads + tid;
      const bool pass = c < nc && lex_less(s[u], (int)c, thr_d, thr_i);
      const unsigned long long m = __ballot(pass);
      if (m) {  // one LDS atomic per wave: slots by prefix count of the ballot
        int base = 0;
        if ((tid & 63) == __builtin_ctzll(m)) base = atomicAdd(s_cnt, __popcll(m));
        base = __shfl(base, __builtin_ctzll(m), kWave);
        if (pass) {
          const int slot =
              base + __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                               __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
          bd[slot] = s[u];
          bi[slot] = (int)c;
        }
      }
    }
    __syncthreads();
    const int n = *s_cnt;
    // every wave has read the count before any wave appends the next step's candidates
    // (a late read would see them and could disagree on the compaction below)
    __syncthreads();
    if (n > cap - kWideStep) {  // block-uniform: keep the first kp1, tighten the threshold
      int P = 1;
      while (P < n) P <<= 1;
      block_sort(bd, bi, n, P);
      const int keep = min(n, kp1);
      if (keep == kp1) {
        thr_d = bd[kp1 - 1];
        thr_i = bi[kp1 - 1];
      }
      __syncthreads();  // every thread has read the threshold before s_cnt changes
      if (tid == 0) *s_cnt = keep;
      __syncthreads();
    }
  }
  const int n = *s_cnt;
  int P = 1;
  while (P < n) P <<= 1;
  block_sort(bd, bi, n, P);
  for (int r = tid; r < kp1; r += kWideThreads) {
    a.D[q * kp1 + r] = sqrt_rn(bd[r]);
    if (a.I64) a.I64[q * kp1 + r] = bi[r];
    if (a.I32) a.I32[(int64_t)r * a.nq + q] = bi[r];  // transposed [kp1][nq]
  }
  __syncthreads();  // the buffer is reused by the next query
}

template <bool kTransposed, bool kGlobalBuf>
__global__ __launch_bounds__(kWideThreads) void wide_exact_kernel(ExactArgs a, int cap) {
  extern __shared__ char wide_smem[];
  __shared__ int s_cnt;
  double* bd;
  int* bi;
  if constexpr (kGlobalBuf) {
    bd = a.wbuf_d + (int64_t)blockIdx.x * cap;
    bi = a.wbuf_i + (int64_t)blockIdx.x * cap;
  } else {
    bd = reinterpret_cast<double*>(wide_smem);
    bi = reinterpret_cast<int*>(wide_smem + (size_t)cap * sizeof(double));
  }
  const int count = stage_count(a);
  stage_report(a);
  for (int fi = blockIdx.x; fi < count; fi += gridDim.x)
    wide_query<kTransposed>(a, stage_query(a, fi), stage_bound(a, fi), bd, bi, cap, &s_cnt);
}

template <int LIST>
static void launch_exact_list(const ExactArgs& a, hipStream_t st) {
  // the chunked form's partial lists are sized for kExactGrid blocks
  const unsigned grid =
      a.part_d ? kExactGrid : (unsigned)std::min<int64_t>(std::max<int64_t>(a.nq, 1), 4096);
  hipLaunchKernelGGL((exact_kernel<LIST>), dim3(grid), dim3(256), 0, st, a);
  if (a.part_d) hipLaunchKernelGGL(exact_merge_kernel, dim3(grid), dim3(256), 0, st, a, (int)grid);
}

void launch_exact_stage(const ExactArgs& a, hipStream_t st) {
  if (!a.candT && a.kp1 <= 64) {
    // per-thread list >= kp1
    if (a.kp1 <= 8)
      launch_exact_list<8>(a, st);
    else if (a.kp1 <= 16)
      launch_exact_list<16>(a, st);
    else if (a.kp1 <= 40)
      launch_exact_list<40>(a, st);
    else
      launch_exact_list<64>(a, st);
    return;
  }
  const int cap = wide_cap(a.kp1);
  const dim3 g((unsigned)wide_grid(a.nq, a.all, a.kp1));
  if (cap > kWideLdsCap) {
    if (a.candT)
      hipLaunchKernelGGL((wide_exact_kernel<true, true>), g, dim3(kWideThreads), 0, st, a, cap);
    else
      hipLaunchKernelGGL((wide_exact_kernel<false, true>), g, dim3(kWideThreads), 0, st, a, cap);
    return;
  }
  const size_t lds = (size_t)cap * (sizeof(double) + sizeof(int));
  if (a.candT)
    hipLaunchKernelGGL((wide_exact_kernel<true, false>), g, dim3(kWideThreads), lds, st, a, cap);
  else
    hipLaunchKernelGGL((wide_exact_kernel<false, false>), g, dim3(kWideThreads), lds, st, a, cap);
}

// ---------------------------------------------------------------------------------------
// transposed copy + validation (exhaustive plans)
// ---------------------------------------------------------------------------------------
// A block takes 32 rows and walks their features 64 at a time: the tile is read row-major
// (consecutive threads, consecutive features) and written feature-major (consecutive threads,
// consecutive rows).  Rows holding a NaN / inf coordinate are counted into bad[0]
// (sklearn's check_array).  The f64 scan has no squared-norm limit, so no overflow count.
constexpr int kTrRows = 32;
constexpr int kTrCols = 64;
__global__ __launch_bounds__(256) void transpose_validate_kernel(const float* __restrict__ X,
                                                                 int64_t n, int d,
                                                                 float* __restrict__ XT,
                                                                 unsigned* __restrict__ bad) {
  __shared__ float tile[kTrRows][kTrCols + 1];
  __shared__ unsigned rowbad[kTrRows];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * kTrRows;
  if (tid < kTrRows) rowbad[tid] = 0u;
  for (int f0 = 0; f0 < d; f0 += kTrCols) {
    __syncthreads();
    for (int e = tid; e < kTrRows * kTrCols; e += 256) {
      const int ri = e / kTrCols, fi = e % kTrCols;
      const int64_t r = r0 + ri;
      const int f = f0 + fi;
      float v = 0.f;
      if (r < n && f < d) {
        v = X[r * d + f];
        if (!isfinite(v)) atomicOr(&rowbad[ri], 1u);
      }
      tile[ri][fi] = v;
    }
    __syncthreads();
    if (XT)
      for (int e = tid; e < kTrRows * kTrCols; e += 256) {
        const int fi = e / kTrRows, ri = e % kTrRows;
        const int64_t r = r0 + ri;
        const int f = f0 + fi;
        if (r < n && f < d) XT[(int64_t)f * n + r] = tile[ri][fi];
      }
  }
  __syncthreads();
  if (tid == 0) {
    unsigned c = 0;
    for (int i = 0; i < kTrRows; ++i) c += rowbad[i];
    if (c && bad) atomicAdd(bad, c);
  }
}

void launch_transpose_validate(const float* X, int64_t n, int d, float* candT, unsigned* bad,
                               hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(transpose_validate_kernel, dim3((unsigned)((n + kTrRows - 1) / kTrRows)),
                     dim3(256), 0, st, X, n, d, candT, bad);
}

}  // namespace knn
}  // namespace mepol
