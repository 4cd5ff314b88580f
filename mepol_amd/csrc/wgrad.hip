// Weight gradient of a linear layer over a tall batch, dW = dy^T x (dy [n, O], x [n, I], both
// row-major f64; dW [O, I]): the policy's dW2 = dz2^T h1 (src/policy.py:21-26 Linear, its
// autograd weight gradient at mepol.py:278), K = n = the particle count.
//
// Split-K on the f64 matrix cores with no LDS and no barrier: both operands are read straight
// from L2 into the MFMA fragments, because with K running down the rows each fragment is whole
// cache lines -- v_mfma_f64_16x16x4f64 takes A[m][k] in lane (m = l & 15, k = l >> 4) and
// B[k][n] in lane (k, n = l & 15), i.e. dy[r0 + k][o0 + m] and x[r0 + k][i0 + n]: four rows of
// 16 consecutive doubles (4 x 128 B) per wave-instruction.  One wave owns a 64 (o) x 80 (i)
// output block (20 accumulators) over one K-slice, with the fragments of the next k-step
// in flight; the K-slices' partial blocks are summed in a fixed order by a second launch (the
// same bits every run).  The tiles of one K-slice are dispatched back to back onto one XCD, so
// its rows come from HBM once and from that XCD's L2 for the other tiles.
//
// Replaces rocBLAS's split-K bmm + torch.sum (policy._weight_grad) on the off-policy
// iteration's dW2: 1.04 ms + reduce at C3 (46 TF/s on 48 GF).
#include "common.hpp"

#include <algorithm>

namespace mepol {
namespace wgrad {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int FO = 4, FI = 5;      // 16 x 16 fragments per wave: 64 (o) x 80 (i)
constexpr int kOcc = 2;            // waves per SIMD (VGPR budget 256)
constexpr int BO = 16 * FO, BI = 16 * FI;
constexpr int NL = FO + FI;        // operand loads per lane and k-step
// k-steps of operands in the register ring (3 spills at this tile).  Measured slower
// (tools/wgrad_probe.py, profiles/r5/f64/wgrad_probe.txt): 64 x 64 tiles with 3 stages, and
// 80 x 80 tiles at one wave per SIMD with 2 or 3 stages.
constexpr int NS = 2;
constexpr int kMaxSlices = 128;
constexpr int kSliceRowsMin = 256;

// K-slices: enough (tile, slice) waves for one full round on the 1024 SIMDs at the kernel's
// occupancy, in multiples of 8 (the slice -> XCD map below has no idle blocks), and no slice
// shorter than kSliceRowsMin rows.
inline int slices_for(int64_t n, int O, int I) {
  const int64_t ntile = (int64_t)((O + BO - 1) / BO) * ((I + BI - 1) / BI);
  int64_t s = std::max<int64_t>(8, 1024 * kOcc / ntile);
  s = std::min<int64_t>(s, std::max<int64_t>(8, n / kSliceRowsMin));
  return (int)std::min<int64_t>(kMaxSlices, s & ~7);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kOcc))) void wgrad_kernel(
    const double* __restrict__ dy, int64_t n, int O, const double* __restrict__ x, int I,
    int nob, int nib, int S, int64_t slice_rows, double* __restrict__ part) {
  // block b -> (slice, tile): blocks b and b + 8 share an XCD under the round-robin dispatch,
  // so XCD b % 8 runs slices xcd, xcd + 8, ... with the ntile tiles of each back to back
  const int ntile = nob * nib;
  const int64_t b = blockIdx.x;
  const int64_t j = b >> 3;
  const int64_t s = (j / ntile) * 8 + (b & 7);
  const int tile = (int)(j % ntile);
  if (s >= S) return;
  const int ob = tile / nib, ib = tile % nib;
  const int l = threadIdx.x, fr = l & 15, g = l >> 4;
  const int64_t r_begin = s * slice_rows;
  const int64_t r_end = min(n, r_begin + slice_rows);
  if (r_begin >= r_end) {  // an empty slice still owns its partial block: zeros
    for (int t = 0; t < FO; ++t)
      for (int q = 0; q < 4; ++q) {
        const int o = ob * BO + 16 * t + g + 4 * q;
        for (int u = 0; u < FI; ++u) {
          const int i = ib * BI + 16 * u + fr;
          if (o < O && i < I) part[((int64_t)s * O + o) * I + i] = 0.0;
        }
      }
    return;
  }
  // this lane's columns (clamped: columns past O / I only feed outputs that are not stored)
  int oc[FO], ic[FI];
#pragma unroll
  for (int t = 0; t < FO; ++t) oc[t] = min(ob * BO + 16 * t + fr, O - 1);
#pragma unroll
  for (int u = 0; u < FI; ++u) ic[u] = min(ib * BI + 16 * u + fr, I - 1);

  d4 acc[FO][FI];
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int u = 0; u < FI; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};

  double R[NS][NL];
  // k-step ks reads rows r_begin + 4 ks + (0..3); rows past the slice are clamped here and
  // zeroed at use (only the last k-step can hold them)
  auto load = [&](double (&D)[NL], int64_t ks) __attribute__((always_inline)) {
    const int64_t r = min(r_begin + 4 * ks + g, r_end - 1);
    const double* yr = dy + r * O;
    const double* xr = x + r * I;
#pragma unroll
    for (int t = 0; t < FO; ++t) D[t] = yr[oc[t]];
#pragma unroll
    for (int u = 0; u < FI; ++u) D[FO + u] = xr[ic[u]];
  };
  auto mma = [&](const double (&D)[NL]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < FO; ++t)
#pragma unroll
      for (int u = 0; u < FI; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(D[t], D[FO + u], acc[t][u], 0, 0, 0);
  };
  const int64_t rows = r_end - r_begin;
  const int64_t nfull = rows / 4;               // k-steps with 4 rows in the slice
  const int64_t nks = (rows + 3) / 4;
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) load(R[p], min<int64_t>(p, nks - 1));
  int64_t ks = 0;
  // steady state, unrolled by NS (compile-time ring slots): k-step ks is in R[ks % NS]
#pragma nounroll
  for (; ks + NS <= nfull; ks += NS) {
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      load(R[(p + NS - 1) % NS], min<int64_t>(ks + p + NS - 1, nks - 1));
      mma(R[p]);
    }
  }
  // the remaining (< NS) full k-steps and the ragged last one, in the same ring rotation
#pragma unroll
  for (int p = 0; p < NS; ++p) {
    if (ks + p < nks) {  // uniform
      if (ks + p + NS - 1 < nks) load(R[(p + NS - 1) % NS], ks + p + NS - 1);
      if (ks + p >= nfull) {  // ragged: rows past the slice end contribute zero
        const bool ok = r_begin + 4 * (ks + p) + g < r_end;
#pragma unroll
        for (int v = 0; v < NL; ++v) R[p][v] = ok ? R[p][v] : 0.0;
      }
      mma(R[p]);
    }
  }
  // C/D map of the f64 16x16x4 MFMA: col = lane & 15, row = (lane >> 4) + 4 q
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int o = ob * BO + 16 * t + g + 4 * q;
#pragma unroll
      for (int u = 0; u < FI; ++u) {
        const int i = ib * BI + 16 * u + fr;
        if (o < O && i < I) part[((int64_t)s * O + o) * I + i] = acc[t][u][q];
      }
    }
}

// out[e] = sum over the slices s = 0..S-1 of part[s][e], in that order; the loads of eight
// slices are in flight at once (S is a multiple of 8), the adds stay sequential
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const double* __restrict__ part, int S,
                                                          int64_t elems, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= elems) return;
  double v = 0.0;
  for (int s = 0; s < S; s += 8) {
    double p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = part[(int64_t)(s + u) * elems + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += p[u];
  }
  out[e] = v;
}

}  // namespace wgrad
}  // namespace mepol

extern "C" int mepol_weight_grad_workspace_size(int64_t n, int out_features, int in_features,
                                                size_t* bytes) {
  if (!bytes || n < 0 || out_features <= 0 || in_features <= 0) return mepol::kErrBadArg;
  *bytes = (size_t)mepol::wgrad::slices_for(n, out_features, in_features) * out_features *
           in_features * sizeof(double);
  return 0;
}

extern "C" int mepol_weight_grad(const double* dy, int64_t n, int out_features, const double* x,
                                 int in_features, double* dW, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  using namespace mepol::wgrad;
  const int O = out_features, I = in_features;
  if (n <= 0 || O <= 0 || I <= 0 || !dy || !x || !dW || !workspace) {
    mepol::set_error("mepol_weight_grad: bad arguments");
    return mepol::kErrBadArg;
  }
  const int S = slices_for(n, O, I);
  const size_t need = (size_t)S * O * I * sizeof(double);
  if (workspace_bytes < need) {
    mepol::set_error("mepol_weight_grad: workspace %zu < %zu", workspace_bytes, need);
    return mepol::kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  const int nob = (O + BO - 1) / BO, nib = (I + BI - 1) / BI;
  const int64_t slice_rows = ((n + S - 1) / S + 3) / 4 * 4;  // whole k-steps but the last
  const unsigned blocks = (unsigned)((int64_t)S * nob * nib);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(wgrad_kernel, dim3(blocks), dim3(64), 0, st, dy, n, O, x, I, nob, nib, S,
                     slice_rows, part);
  MEPOL_CHECK_LAUNCH();
  const int64_t elems = (int64_t)O * I;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)((elems + 255) / 256)), dim3(256), 0, st,
                     part, S, elems, dW);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
