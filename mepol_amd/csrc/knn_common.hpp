// Shared pieces of the k-NN translation units (knn.hip: pack / refine / exact / dispatch;
// knn_select_ks{1..4}.hip: the selection kernels, one TU per k-step count so they build in
// parallel).  See knn.hip for the pipeline.
#pragma once
#include "common.hpp"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdlib>

namespace mepol {
namespace knn {

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;


constexpr int kMaxSplit = 16;
constexpr int kExactGrid = 512;    // blocks of the exhaustive fallback (exact_kernel)
constexpr int kRefineList = 64;    // approximate candidates refine ranks per query (one wave)

// ---------------------------------------------------------------------------------------
// 2. select: list helpers
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

template <int LIST>
__device__ __forceinline__ float list_at(const float (&ld)[LIST], int j) {
  float v = INFINITY;
#pragma unroll
  for (int i = 0; i < LIST; ++i) v = (i == j) ? ld[i] : v;
  return v;
}

// LDS byte address of a __shared__ object (the M0 operand of an LDS-DMA load); wave-uniform.
template <typename T>
__device__ __forceinline__ unsigned lds_addr(T* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(__attribute__((address_space(3))) T*)(p));
}

// Row (candidate within the tile) of accumulator register r for lane l (32x32 C/D map).
__device__ __forceinline__ int acc_row(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }

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

__device__ __forceinline__ void split_f16(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);  // v - hi is exact in f32
}

// probe seeds (knn_select.hpp, probe16_kernel): sampled candidate tiles per query, and which
// smallest tile minimum of a lane becomes the seed
constexpr int kProbeTiles = 256;
constexpr int kProbeKth = 8;

constexpr float kPadNorm16 = 60000.f;  // scaled |c|^2 of padding candidates (> any real D')

// Arguments of the selection launch (make_plan's fields the select kernels read).
struct SelectArgs {
  const _Float16* apack;
  const float* query;
  int64_t nq;
  int d;
  int64_t nct;
  int split;
  int64_t tiles_per_split;
  int keep;
  int LIST16;
  int nh;
  int64_t nqt;
  const unsigned* scal;
  float* out_v;
  int* out_i;
  int* seed;  // [nq] ordered keys of the per-query prune bounds the ranges publish (nullable)
  int probe;  // seed from the probe sample first (probe16_kernel; needs seed)
};

// Order-preserving map of a float to an int (atomicMin on the int orders like the float; the
// selection values are |c|^2 - 2 c.q, which can be negative).
__device__ __forceinline__ int float_order_key(float v) {
  const int b = __float_as_int(v);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float order_key_float(int k) {
  return __int_as_float(k >= 0 ? k : k ^ 0x7fffffff);
}
constexpr int kSeedNone = 0x7f800000;  // float_order_key(+inf)

// knn_select_ks<KS16>.hip
template <int KS16>
void launch_select(const SelectArgs& a, hipStream_t st);

// ---------------------------------------------------------------------------------------
// exact f64 arithmetic shared by refine (knn.hip) and the exhaustive stage (knn_exact.hip)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ bool lex_less(double a, int ai, double b, int bi) {
  return a < b || (a == b && ai < bi);
}

// Exact f64 squared distance, summed in feature order with no contraction (matches the
// reference's kd_tree rdist: sum of (x_f - y_f)^2 in double, f = 0..d-1).
// The row is read 32 features at a time with every load issued before the first use (clamped,
// unconditional addresses): one memory latency per chunk instead of one per feature.
__device__ __forceinline__ double exact_d2(const float* __restrict__ a, const float* __restrict__ b,
                                           int d) {
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

// ---------------------------------------------------------------------------------------
// 4. the exhaustive stage (knn_exact.hip)
// ---------------------------------------------------------------------------------------
// Which queries the stage answers: the queue refine filled (flag_count / flag_list), or every
// query -- a plan that screens nothing (exhaustive plans) or an input the f16 screen cannot
// scale (a squared norm beyond f32: scal[5] != 0; the f64 scan has no such limit).  Nothing
// at all when the input was rejected (scal[4]: a NaN / inf coordinate).
struct ExactArgs {
  const float* cand;      // [nc][d] row-major (the caller's input)
  const float* candT;     // [d][nc] transposed copy (exhaustive plans; nullable)
  int64_t nc;
  const float* query;     // [nq][d]
  int64_t nq;
  int d;
  int kp1;
  int* flag_count;        // queued queries (refine); set to nq when scal[5] sends all
  const int* flag_list;
  const unsigned* scal;   // [4]: rejected rows, [5]: rows beyond the f16 screen
  int all;                // 1: every query (exhaustive plan)
  double* D;
  int64_t* I64;
  int32_t* I32;           // transposed [kp1][nq]
  double* part_d;         // chunked register-list form: kExactGrid partial lists (nullable)
  int* part_i;
  double* wbuf_d;         // block-select form, lists beyond LDS: grid x cap entries (nullable)
  int* wbuf_i;
  // per queued query (flag_list order): an upper bound on its (k+1)-th exact squared distance,
  // the (k+1)-th smallest exact d^2 refine evaluated (nullable; unused when every query runs)
  const double* flag_bound;
};

// Block-select capacity (entries) for kp1: room for kp1 plus one step of every thread.
int wide_cap(int kp1);
// Blocks and global-buffer bytes of the block-select form (all = every query of nq).
int wide_grid(int64_t nq, int all, int kp1);
size_t wide_buffer_bytes(int64_t nq, int all, int kp1);
// Launches the stage: register lists for kp1 <= 64 over row-major candidates, the block-select
// form otherwise and whenever a transposed copy is given.
void launch_exact_stage(const ExactArgs& a, hipStream_t st);
// candT <- cand transposed ([d][n]; nullable: validation only); bad[0] += rows holding a NaN / inf.
void launch_transpose_validate(const float* X, int64_t n, int d, float* candT, unsigned* bad,
                               hipStream_t st);

}  // namespace knn
}  // namespace mepol
