// First policy layer (Linear(nf, h0) + ReLU of GaussianPolicy.net, src/policy.py:21-26) for the
// large-batch off-policy passes: fused forward h = relu(x W^T + b) and the backward of the
// weights (dW = (dh * [h > 0])^T x, db = sum dh * [h > 0]).  The input width nf is small
// (2 for MountainCar/GridWorld, 29 for Ant), so this layer is pure streaming of the N x h0
// activation; rocBLAS + separate bias/ReLU/threshold kernels move it three times as often.
//
// Mapping: a wave owns 64 consecutive output columns (one per lane: coalesced 512-B row
// segments) and a strided set of rows; the row's nf inputs are wave-uniform (scalar loads),
// the lane's weight row lives in VGPRs.  Row reductions go through fixed-order partials.
#include "common.hpp"

#include <algorithm>
#include <map>
#include <mutex>
#include <utility>

namespace mepol {
namespace mlp {

constexpr int kChunk = 64;  // rows staged per block iteration
constexpr int kThreads = 256;

// Stage kChunk rows of x (contiguous kChunk*F doubles) into LDS with coalesced loads; features
// [F, FP) stay zero so the unrolled FMA chain needs no per-feature guard.  Several blocks per CU
// overlap one block's staging with the others' compute.
template <int FP>
__device__ __forceinline__ void stage_rows(const double* __restrict__ x, int F, int nrow,
                                           int64_t r0, double (*sx)[FP]) {
  const double* src = x + r0 * F;
  for (int e = threadIdx.x; e < nrow * F; e += kThreads) {
    const int rr = e / F;
    sx[rr][e - rr * F] = src[e];
  }
}

template <int FP>
__global__ __launch_bounds__(kThreads) void layer_fwd_kernel(const double* __restrict__ x,
                                                             int64_t N, int F,
                                                             const double* __restrict__ W,
                                                             const double* __restrict__ b, int H,
                                                             double* __restrict__ h) {
  __shared__ double sx[kChunk][FP];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + l;
  const bool col = c < H;
  double wr[FP];
#pragma unroll
  for (int f = 0; f < FP; ++f) wr[f] = (col && f < F) ? W[(int64_t)c * F + f] : 0.0;
  const double bc = col ? b[c] : 0.0;
  for (int e = threadIdx.x; e < kChunk * FP; e += kThreads) sx[e / FP][e % FP] = 0.0;
  const int64_t step = (int64_t)gridDim.x * kChunk;
  for (int64_t r0 = (int64_t)blockIdx.x * kChunk; r0 < N; r0 += step) {
    const int nrow = (int)min<int64_t>(kChunk, N - r0);
    __syncthreads();
    stage_rows<FP>(x, F, nrow, r0, sx);
    __syncthreads();
#pragma unroll 1
    for (int rr = w; rr < nrow; rr += 4) {
      double acc = bc;
#pragma unroll
      for (int f = 0; f < FP; ++f) acc = fma(sx[rr][f], wr[f], acc);
      if (col) h[(r0 + rr) * H + c] = fmax(acc, 0.0);
    }
  }
}

// part: [gridDim.x][H][F + 1]  (dW row c then db_c)
template <int FP>
__global__ __launch_bounds__(kThreads) void layer_bwd_kernel(const double* __restrict__ dh,
                                                             const double* __restrict__ h,
                                                             const double* __restrict__ x,
                                                             int64_t N, int F, int H,
                                                             double* __restrict__ part) {
  constexpr int kRows = 4;  // rows of h/dh in flight per wave
  __shared__ double sx[kChunk][FP];
  __shared__ double sacc[64][FP + 1];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + l;
  const bool col = c < H;
  const int cc = col ? c : H - 1;  // clamped column: loads stay in bounds, results discarded
  double acc[FP], accb = 0.0;
#pragma unroll
  for (int f = 0; f < FP; ++f) acc[f] = 0.0;
  for (int e = threadIdx.x; e < kChunk * FP; e += kThreads) sx[e / FP][e % FP] = 0.0;
  const int64_t step = (int64_t)gridDim.x * kChunk;
  for (int64_t r0 = (int64_t)blockIdx.x * kChunk; r0 < N; r0 += step) {
    const int nrow = (int)min<int64_t>(kChunk, N - r0);
    __syncthreads();
    stage_rows<FP>(x, F, nrow, r0, sx);
    __syncthreads();
#pragma unroll 1
    for (int rb = w * kRows; rb < nrow; rb += 4 * kRows) {
      double hv[kRows], dv[kRows];
#pragma unroll
      for (int q = 0; q < kRows; ++q) {
        const int rr = min(rb + q, nrow - 1);
        const int64_t o = (r0 + rr) * H + cc;
        hv[q] = h[o];
        dv[q] = dh[o];
      }
#pragma unroll
      for (int q = 0; q < kRows; ++q) {
        const double dz = (col && rb + q < nrow && hv[q] > 0.0) ? dv[q] : 0.0;
#pragma unroll
        for (int f = 0; f < FP; ++f) acc[f] = fma(dz, sx[min(rb + q, kChunk - 1)][f], acc[f]);
        accb += dz;
      }
    }
  }
  // Fixed-order cross-wave sum: wave 0 writes, waves 1..3 add in turn.
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int f = 0; f < FP; ++f) sacc[l][f] = (ww == 0) ? acc[f] : sacc[l][f] + acc[f];
      sacc[l][FP] = (ww == 0) ? accb : sacc[l][FP] + accb;
    }
    __syncthreads();
  }
  if (w == 0 && col) {
    double* rec = part + ((int64_t)blockIdx.x * H + c) * (F + 1);
    for (int f = 0; f < F; ++f) rec[f] = sacc[l][f];
    rec[F] = sacc[l][FP];
  }
}

// dW[c][f] = sum_b part[b][c][f], db[c] = sum_b part[b][c][F]; fixed order.
__global__ void layer_reduce_kernel(const double* __restrict__ part, int nb, int H, int F,
                                    double* __restrict__ dW, double* __restrict__ db) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = (int64_t)H * (F + 1);
  if (e >= m) return;
  double s = 0.0;
  for (int b = 0; b < nb; ++b) s += part[(int64_t)b * m + e];
  const int c = (int)(e / (F + 1)), f = (int)(e % (F + 1));
  if (f < F)
    dW[(int64_t)c * F + f] = s;
  else if (db)
    db[c] = s;
}

constexpr int kRowBlocks = 256;  // upper bound on row-chunk blocks per column tile

// Blocks per column tile so that the whole grid is resident at once (no partial second wave of
// blocks): CUs x resident blocks per CU / column tiles, capped by kRowBlocks and the chunks.
// The device queries are cached (first call per kernel/device), so launches made under HIP
// graph capture issue no runtime queries.
template <typename Kernel>
int row_blocks(Kernel kernel, int64_t n, int col_tiles) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;  // (kernel, device) -> CUs x blocks
  int dev = 0;
  (void)hipGetDevice(&dev);
  int resident;
  {
    std::lock_guard<std::mutex> lock(mu);
    auto key = std::make_pair((const void*)kernel, dev);
    auto it = cache.find(key);
    if (it == cache.end()) {
      int cus = 256, per_cu = 1;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) !=
              hipSuccess ||
          per_cu < 1)
        per_cu = 1;
      it = cache.emplace(key, cus * per_cu).first;
    }
    resident = it->second;
  }
  const int64_t chunks = std::max<int64_t>((n + kChunk - 1) / kChunk, 1);
  const int64_t fit = std::max<int64_t>((int64_t)resident / col_tiles, 1);
  return (int)std::min<int64_t>(std::min<int64_t>(fit, kRowBlocks), chunks);
}

}  // namespace mlp
}  // namespace mepol

using namespace mepol;
using namespace mepol::mlp;

#define MEPOL_FP_SWITCH(F, CALL)      \
  if ((F) <= 2) {                     \
    constexpr int FP = 2;             \
    CALL;                             \
  } else if ((F) <= 4) {              \
    constexpr int FP = 4;             \
    CALL;                             \
  } else if ((F) <= 8) {              \
    constexpr int FP = 8;             \
    CALL;                             \
  } else if ((F) <= 16) {             \
    constexpr int FP = 16;            \
    CALL;                             \
  } else if ((F) <= 32) {             \
    constexpr int FP = 32;            \
    CALL;                             \
  } else {                            \
    constexpr int FP = 64;            \
    CALL;                             \
  }

extern "C" int mepol_layer_forward(const double* x, int64_t n, int in_features, const double* W,
                                   const double* b, int out_features, double* h_out,
                                   void* stream) {
  if (n < 0 || in_features <= 0 || in_features > 64 || out_features <= 0 || !x || !W || !b ||
      !h_out) {
    set_error("mepol_layer_forward: bad arguments (in_features <= 64)");
    return kErrBadArg;
  }
  if (n == 0) return 0;
  const int gy = (out_features + 63) / 64;
  hipStream_t st = (hipStream_t)stream;
  MEPOL_FP_SWITCH(in_features, {
    const int gx = row_blocks(layer_fwd_kernel<FP>, n, gy);
    hipLaunchKernelGGL((layer_fwd_kernel<FP>), dim3(gx, gy), dim3(kThreads), 0, st, x, n,
                       in_features, W, b, out_features, h_out);
  });
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_layer_workspace_size(int64_t n, int in_features, int out_features,
                                          size_t* bytes) {
  if (!bytes || in_features <= 0 || out_features <= 0) return kErrBadArg;
  const int gx = (int)std::min<int64_t>(kRowBlocks, std::max<int64_t>((n + kChunk - 1) / kChunk, 1));
  *bytes = (size_t)gx * out_features * (in_features + 1) * sizeof(double);
  return 0;
}

// dW [out, in], db [out] (nullable) of relu(x W^T + b) given dh = dL/dh and the forward output h.
extern "C" int mepol_layer_backward(const double* dh, const double* h, const double* x, int64_t n,
                                    int in_features, int out_features, double* dW, double* db,
                                    void* workspace, size_t workspace_bytes, void* stream) {
  if (n <= 0 || in_features <= 0 || in_features > 64 || out_features <= 0 || !dh || !h || !x ||
      !dW || !workspace) {
    set_error("mepol_layer_backward: bad arguments");
    return kErrBadArg;
  }
  const int gy = (out_features + 63) / 64;
  int gx = 1;
  MEPOL_FP_SWITCH(in_features, gx = row_blocks(layer_bwd_kernel<FP>, n, gy));
  const size_t need = (size_t)gx * out_features * (in_features + 1) * sizeof(double);
  if (workspace_bytes < need) {
    set_error("mepol_layer_backward: workspace %zu < %zu", workspace_bytes, need);
    return kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
  MEPOL_FP_SWITCH(in_features,
                  hipLaunchKernelGGL((layer_bwd_kernel<FP>), dim3(gx, gy), dim3(kThreads), 0, st,
                                     dh, h, x, n, in_features, out_features, part));
  MEPOL_CHECK_LAUNCH();
  const int64_t m = (int64_t)out_features * (in_features + 1);
  hipLaunchKernelGGL(layer_reduce_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, part,
                     gx, out_features, in_features, dW, db);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
