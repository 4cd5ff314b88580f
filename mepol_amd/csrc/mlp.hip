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

namespace mepol {
namespace mlp {

template <int FP>
__global__ __launch_bounds__(256) void layer_fwd_kernel(const double* __restrict__ x, int64_t N,
                                                        int F, const double* __restrict__ W,
                                                        const double* __restrict__ b, int H,
                                                        double* __restrict__ h) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + l;
  const bool col = c < H;
  double wr[FP];
#pragma unroll
  for (int f = 0; f < FP; ++f) wr[f] = (col && f < F) ? W[(int64_t)c * F + f] : 0.0;
  const double bc = col ? b[c] : 0.0;
  const int64_t stride = (int64_t)gridDim.x * 4;
  const int64_t r0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + w));
  for (int64_t r = r0; r < N; r += stride) {
    const double* xr = x + r * F;  // wave-uniform address -> scalar loads
    double acc = bc;
#pragma unroll
    for (int f = 0; f < FP; ++f)
      if (f < F) acc = fma(xr[f], wr[f], acc);
    if (col) h[r * H + c] = fmax(acc, 0.0);
  }
}

// part: [gridDim.x][H][F + 1]  (dW row c then db_c)
template <int FP>
__global__ __launch_bounds__(256) void layer_bwd_kernel(const double* __restrict__ dh,
                                                        const double* __restrict__ h,
                                                        const double* __restrict__ x, int64_t N,
                                                        int F, int H, double* __restrict__ part) {
  __shared__ double sacc[4][64][FP + 1];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + l;
  const bool col = c < H;
  double acc[FP], accb = 0.0;
#pragma unroll
  for (int f = 0; f < FP; ++f) acc[f] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 4;
  const int64_t r0 = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + w));
  for (int64_t r = r0; r < N; r += stride) {
    double dz = 0.0;
    if (col) {
      const double hv = h[r * H + c];
      dz = (hv > 0.0) ? dh[r * H + c] : 0.0;
    }
    const double* xr = x + r * F;
#pragma unroll
    for (int f = 0; f < FP; ++f)
      if (f < F) acc[f] = fma(dz, xr[f], acc[f]);
    accb += dz;
  }
#pragma unroll
  for (int f = 0; f < FP; ++f) sacc[w][l][f] = acc[f];
  sacc[w][l][FP] = accb;
  __syncthreads();
  if (w == 0 && col) {
    double* rec = part + ((int64_t)blockIdx.x * H + c) * (F + 1);
    for (int f = 0; f < F; ++f)
      rec[f] = ((sacc[0][l][f] + sacc[1][l][f]) + sacc[2][l][f]) + sacc[3][l][f];
    rec[F] = ((sacc[0][l][FP] + sacc[1][l][FP]) + sacc[2][l][FP]) + sacc[3][l][FP];
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

constexpr int kRowBlocks = 128;  // blocks along the rows (x 4 waves): 512 row streams per column tile

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
  const int gx = (int)std::min<int64_t>(kRowBlocks, (n + 3) / 4);
  dim3 g(gx, (out_features + 63) / 64);
  hipStream_t st = (hipStream_t)stream;
  MEPOL_FP_SWITCH(in_features, hipLaunchKernelGGL((layer_fwd_kernel<FP>), g, dim3(256), 0, st, x,
                                                  n, in_features, W, b, out_features, h_out));
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_layer_workspace_size(int64_t n, int in_features, int out_features,
                                          size_t* bytes) {
  if (!bytes || in_features <= 0 || out_features <= 0) return kErrBadArg;
  const int gx = (int)std::min<int64_t>(kRowBlocks, std::max<int64_t>((n + 3) / 4, 1));
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
  const int gx = (int)std::min<int64_t>(kRowBlocks, (n + 3) / 4);
  const size_t need = (size_t)gx * out_features * (in_features + 1) * sizeof(double);
  if (workspace_bytes < need) {
    set_error("mepol_layer_backward: workspace %zu < %zu", workspace_bytes, need);
    return kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  dim3 g(gx, (out_features + 63) / 64);
  double* part = (double*)workspace;
  MEPOL_FP_SWITCH(in_features, hipLaunchKernelGGL((layer_bwd_kernel<FP>), g, dim3(256), 0, st, dh,
                                                  h, x, n, in_features, out_features, part));
  MEPOL_CHECK_LAUNCH();
  const int64_t m = (int64_t)out_features * (in_features + 1);
  hipLaunchKernelGGL(layer_reduce_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, part,
                     gx, out_features, in_features, dW, db);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
