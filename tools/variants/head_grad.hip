// MEASURED AND DROPPED (round 4; not built into the product library).  The graph iteration with
// this backward took 5.46 ms at C3 against 3.77 ms for head_bwd_kernel + rocBLAS dW2 + the dh1
// kernel reading dz2 (profiles/r4/fused_head_dropped_timeline_C3.txt): dw2_kernel 2.22 ms (the
// rocBLAS GEMM 1.0 ms), the dz2-forming dh1 variant 3.93 ms (1.93 ms reading dz2: the formation
// sits between the MFMA block and the barrier of its single workgroup per CU), the record
// reduction 153 us.  Kept as the starting point for a later attempt.
//
// Policy-head backward without the dz2 round trip (round 4).
//
// The reference's loss.backward() (src/algorithms/mepol.py:278) runs through
// GaussianPolicy.get_log_p (src/policy.py:43-51): mu = relu(z2 + b2) Wm^T + bm, logp from mu.
// With dlogp = dH/dlogp per particle (the entropy reverse scan) and, per row n,
//   c[n][a]  = dlogp_n (act_na - mu_na) / sigma_a^2                        (= dL/dmu_na)
//   dz2[n][i] = [z2[n][i] + b2[i] > 0] sum_a c[n][a] Wm[a][i]               (ReLU backward)
// the parameter gradients are
//   dbm[a] = sum_n c[n][a],  dlog_std[a] = sum_n dlogp_n (-1 + (act-mu)^2 e^ls / sigma^3),
//   dWm[a][i] = sum_n c[n][a] relu(z2 + b2)[n][i],  db2[i] = sum_n dz2[n][i],
//   dW2[i][j] = sum_n dz2[n][i] h1[n][j]
// (and dW1 / db1 through dh1 = dz2 W2: gemm.hip, which forms dz2 the same way).  Round 3 wrote
// dz2 (N x 300 f64, 480 MB at C3) in head_bwd_kernel and read it back in a rocBLAS dW2 GEMM and
// the dh1 kernel.  Here dz2 is never written:
//   head_coef_kernel  c [N x A] (12.8 MB at C3) + per-block partials of dbm / dlog_std;
//   dw2_kernel        split-K over rows on the f64 matrix cores: per 16-row k-tile the block
//                     forms its 64 columns of dz2 (and relu(z2 + b2)) from z2, c, Wm, b2 into
//                     LDS and accumulates dW2 (with a column of ones appended to h1: db2) and,
//                     in the first column block, dWm;
//   grad_reduce_kernel  fixed-order sums of the per-chunk records (bitwise reproducible).
// dz2 is formed with head_bwd_kernel's arithmetic (dh = fma(c_a, Wm_a, dh) for a = 0..A-1, then
// the mask), so the values entering the GEMMs are the ones round 3 wrote to HBM.
#include "common.hpp"

#include <algorithm>

namespace mepol {
namespace hgrad {

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr double kStdEps = 1e-7;  // src/utils/dtypes.py:7 (as head.hip)
constexpr int kMaxA = 8;          // fused path: action_dim <= 8 (MC 1, GW 2, Ant 8)
constexpr int kCoefBlocks = 256;  // head_coef_kernel grid (fixed: partial records)

// c[n][a] and per-block partials [blk][2A] = (sum c, sum dlog_std terms), rows grid-strided in
// a fixed order.
__global__ __launch_bounds__(256) void head_coef_kernel(const double* __restrict__ gl,
                                                        const double* __restrict__ act,
                                                        const double* __restrict__ mu,
                                                        const double* __restrict__ log_std,
                                                        int64_t N, int A,
                                                        double* __restrict__ coef,
                                                        double* __restrict__ part) {
  __shared__ double sInv[kMaxA], sEs3[kMaxA];
  __shared__ double sRed[4][2 * kMaxA];
  if (threadIdx.x < kMaxA) {
    const int a = threadIdx.x;
    const double e = a < A ? exp(log_std[a]) : 1.0;
    const double sd = e + kStdEps;
    sInv[a] = 1.0 / (sd * sd);
    sEs3[a] = e / (sd * sd * sd);
  }
  __syncthreads();
  double sb[kMaxA], sl[kMaxA];
#pragma unroll
  for (int a = 0; a < kMaxA; ++a) sb[a] = sl[a] = 0.0;
  for (int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; n < N;
       n += (int64_t)gridDim.x * blockDim.x) {
    const double g = gl[n];
#pragma unroll
    for (int a = 0; a < kMaxA; ++a) {
      if (a < A) {
        const double d = act[n * A + a] - mu[n * A + a];
        const double c = g * d * sInv[a];  // head_bwd_kernel's dm[a]
        coef[n * A + a] = c;
        sb[a] += c;
        sl[a] += g * (-1.0 + d * d * sEs3[a]);
      }
    }
  }
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < kMaxA; ++a) {
    const double x = wave_sum(sb[a]), y = wave_sum(sl[a]);
    if (l == 0) {
      sRed[w][a] = x;
      sRed[w][kMaxA + a] = y;
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * A) {
    const int e = threadIdx.x, a = e % A, which = e / A;
    const int s = which * kMaxA + a;
    part[(int64_t)blockIdx.x * 2 * A + e] = ((sRed[0][s] + sRed[1][s]) + sRed[2][s]) + sRed[3][s];
  }
}

// ---- dW2 / db2 / dWm, split-K over rows ------------------------------------------------------
constexpr int kIB = 64;            // dz2 columns per block (4 waves x one 16-column fragment)
constexpr int kJW = 112;           // h1 columns (+ the ones column) per block: 7 fragments
constexpr int kJF = kJW / 16;
constexpr int kKT = 16;            // rows per LDS k-tile (4 MFMA k-steps)
constexpr int kRowsPerBlock = 4096;
constexpr int kPI = kIB + 2, kPJ = kJW + 2;     // LDS row strides (doubles)
constexpr int kHL = (kKT * kJW + 255) / 256;    // h1 tile elements per thread (13)

// Record per row chunk: [dW2 with db2 as column H0: H1 x (H0 + 1)] [dWm: A x H1].
__global__ __launch_bounds__(256) void dw2_kernel(
    const double* __restrict__ z2, const double* __restrict__ b2, const double* __restrict__ coef,
    const double* __restrict__ Wm, const double* __restrict__ h1, int64_t N, int H1, int H0,
    int A, double* __restrict__ part) {
  __shared__ double sDZ[kKT][kPI];
  __shared__ double sX2[kKT][kPI];
  __shared__ double sH[kKT][kPJ];
  __shared__ double sC[kKT][16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int ib = blockIdx.x, jb = blockIdx.y, rc = blockIdx.z;
  const int i0 = ib * kIB, j0 = jb * kJW;
  const bool dwm = jb == 0;  // the first column block also accumulates dWm
  const int64_t n0 = (int64_t)rc * kRowsPerBlock;
  const int64_t n1 = std::min<int64_t>(N, n0 + kRowsPerBlock);
  // dz2 tile element of this thread: column ci, rows w + 4u (u < 4)
  const int ci = tid & 63, icol = i0 + ci;
  const bool iok = icol < H1;
  double wcol[kMaxA];
#pragma unroll
  for (int a = 0; a < kMaxA; ++a) wcol[a] = (iok && a < A) ? Wm[a * H1 + icol] : 0.0;
  const double bcol = iok ? b2[icol] : 0.0;

  d4 acc[kJF];
#pragma unroll
  for (int f = 0; f < kJF; ++f) acc[f] = d4{0.0, 0.0, 0.0, 0.0};
  d4 accW = d4{0.0, 0.0, 0.0, 0.0};

  // register stage of the next k-tile (loads in flight during the MFMA block): raw z2, the
  // h1 tile and the coefficient rows; dz2 is formed after they land in LDS
  double rz[4], rh[kHL], rcf;
  auto gload = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t n = std::min<int64_t>(k0 + w + 4 * u, n1 - 1);
      rz[u] = z2[n * H1 + (iok ? icol : 0)];
    }
#pragma unroll
    for (int p = 0; p < kHL; ++p) {
      const int e = tid + 256 * p, r = e / kJW, jj = e % kJW, j = j0 + jj;
      const int64_t n = std::min<int64_t>(k0 + (e < kKT * kJW ? r : 0), n1 - 1);
      rh[p] = h1[n * H0 + std::min(j, H0 - 1)];
    }
    {
      const int r = tid >> 4, a = tid & 15;
      const int64_t n = std::min<int64_t>(k0 + r, n1 - 1);
      rcf = coef[n * A + (a < A ? a : 0)];
    }
  };
  auto lstore = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) sX2[w + 4 * u][ci] = rz[u];
#pragma unroll
    for (int p = 0; p < kHL; ++p) {
      const int e = tid + 256 * p;
      if (e < kKT * kJW) {
        const int r = e / kJW, jj = e % kJW, j = j0 + jj;
        const bool ok = k0 + r < n1;
        sH[r][jj] = ok ? (j < H0 ? rh[p] : (j == H0 ? 1.0 : 0.0)) : 0.0;
      }
    }
    {
      const int r = tid >> 4, a = tid & 15;
      sC[r][a] = (a < A && k0 + r < n1) ? rcf : 0.0;
    }
  };
  // dz2 and relu(z2 + b2) of this thread's four elements from the staged z2 and coefficients
  // (head_bwd_kernel's arithmetic); call between two barriers
  auto form = [&](int64_t k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int r = w + 4 * u;
      const bool ok = iok && k0 + r < n1;
      const double zb = sX2[r][ci] + bcol;
      double dh = 0.0;
#pragma unroll
      for (int a = 0; a < kMaxA; ++a)
        if (a < A) dh = fma(sC[r][a], wcol[a], dh);
      sDZ[r][ci] = (ok && zb > 0.0) ? dh : 0.0;
      sX2[r][ci] = ok ? fmax(zb, 0.0) : 0.0;
    }
  };

  if (n0 < n1) {
    gload(n0);
    lstore(n0);
    __syncthreads();
    form(n0);
    __syncthreads();
    for (int64_t k0 = n0; k0 < n1; k0 += kKT) {
      const bool more = k0 + kKT < n1;
      if (more) gload(k0 + kKT);
#pragma nounroll
      for (int s = 0; s < 4; ++s) {
        const double av = sDZ[4 * s + g][16 * w + fr];
#pragma unroll
        for (int f = 0; f < kJF; ++f)
          acc[f] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, sH[4 * s + g][16 * f + fr], acc[f],
                                                        0, 0, 0);
        if (dwm)
          accW = __builtin_amdgcn_mfma_f64_16x16x4f64(sC[4 * s + g][fr],
                                                      sX2[4 * s + g][16 * w + fr], accW, 0, 0, 0);
      }
      __syncthreads();
      if (more) {
        lstore(k0 + kKT);
        __syncthreads();
        form(k0 + kKT);
        __syncthreads();
      }
    }
  }
  // C/D map of the f64 16x16x4 MFMA: col = lane & 15, row = (lane >> 4) + 4 q
  const int64_t m = (int64_t)H1 * (H0 + 1) + (int64_t)A * H1;
  double* rec = part + (int64_t)rc * m;
#pragma unroll
  for (int f = 0; f < kJF; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + 16 * w + g + 4 * q, j = j0 + 16 * f + fr;
      if (i < H1 && j <= H0) rec[(int64_t)i * (H0 + 1) + j] = acc[f][q];
    }
  if (dwm) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int a = g + 4 * q, i = i0 + 16 * w + fr;
      if (a < A && i < H1) rec[(int64_t)H1 * (H0 + 1) + (int64_t)a * H1 + i] = accW[q];
    }
  }
}

// Fixed-order sums: element e of the dW2 records over the row chunks (chunk order), then the
// head_coef partials over its blocks; scattered into dW2 [H1][H0], db2 [H1], dWm [A][H1],
// dbm [A], dlog_std [A].
__global__ __launch_bounds__(256) void grad_reduce_kernel(const double* __restrict__ part,
                                                          int nrc, int H1, int H0, int A,
                                                          const double* __restrict__ cpart,
                                                          int ncb, double* __restrict__ dW2,
                                                          double* __restrict__ db2,
                                                          double* __restrict__ dWm,
                                                          double* __restrict__ dbm,
                                                          double* __restrict__ dls) {
  const int64_t m = (int64_t)H1 * (H0 + 1) + (int64_t)A * H1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e < m) {
    double s = 0.0;
    for (int r = 0; r < nrc; ++r) s += part[(int64_t)r * m + e];
    const int64_t hw = (int64_t)H1 * (H0 + 1);
    if (e < hw) {
      const int i = (int)(e / (H0 + 1)), j = (int)(e % (H0 + 1));
      if (j < H0)
        dW2[(int64_t)i * H0 + j] = s;
      else if (db2)
        db2[i] = s;
    } else {
      dWm[e - hw] = s;
    }
  } else if (e < m + 2 * A) {
    const int k = (int)(e - m);
    double s = 0.0;
    for (int b = 0; b < ncb; ++b) s += cpart[(int64_t)b * 2 * A + k];
    if (k < A)
      dbm[k] = s;
    else
      dls[k - A] = s;
  }
}

inline int64_t row_chunks(int64_t n) { return (n + kRowsPerBlock - 1) / kRowsPerBlock; }

}  // namespace hgrad
}  // namespace mepol

using namespace mepol;
using namespace mepol::hgrad;

// Workspace of the fused head backward: coef [n][a] | coef partials | dW2 records.
extern "C" int mepol_head_grad_workspace_size(int64_t n, int h1w, int h0, int a_dim,
                                              size_t* bytes) {
  if (!bytes || n <= 0 || h1w <= 0 || h0 <= 0 || a_dim <= 0 || a_dim > kMaxA) {
    set_error("mepol_head_grad_workspace_size: bad arguments (action_dim <= %d)", kMaxA);
    return kErrBadArg;
  }
  const int64_t m = (int64_t)h1w * (h0 + 1) + (int64_t)a_dim * h1w;
  *bytes = ((size_t)n * a_dim + (size_t)kCoefBlocks * 2 * a_dim + (size_t)row_chunks(n) * m) *
           sizeof(double);
  return 0;
}

// Stage 1 (the caller's stream, before forking): c = dL/dmu into the workspace and the dbm /
// dlog_std partials.  grad_logp [n], act / mu [n][a_dim], log_std [a_dim].
extern "C" int mepol_head_coef(const double* grad_logp, const double* act, const double* mu,
                               const double* log_std, int64_t n, int a_dim, void* workspace,
                               size_t workspace_bytes, void* stream) {
  if (n <= 0 || a_dim <= 0 || a_dim > kMaxA || !grad_logp || !act || !mu || !log_std ||
      !workspace || workspace_bytes < ((size_t)n * a_dim + (size_t)kCoefBlocks * 2 * a_dim) * 8) {
    set_error("mepol_head_coef: bad arguments");
    return kErrBadArg;
  }
  double* coef = (double*)workspace;
  double* cpart = coef + (size_t)n * a_dim;
  hipLaunchKernelGGL(head_coef_kernel, dim3(kCoefBlocks), dim3(256), 0, (hipStream_t)stream,
                     grad_logp, act, mu, log_std, n, a_dim, coef, cpart);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

// Stage 2 (may run on a forked stream, concurrently with mepol_dh1_layer1_backward_formed):
// dW2 [h1w][h0], db2 [h1w] (nullable), dWm [a][h1w], dbm [a], dlog_std [a] from the forward's
// z2 [n][h1w] (pre-bias), h1 [n][h0], b2, Wm and the coefficients of mepol_head_coef.
extern "C" int mepol_head_dw2(const double* z2, const double* b2, const double* Wm,
                              const double* h1, int64_t n, int h1w, int h0, int a_dim,
                              double* dW2, double* db2, double* dWm, double* dbm,
                              double* dlog_std, void* workspace, size_t workspace_bytes,
                              void* stream) {
  size_t need = 0;
  if (mepol_head_grad_workspace_size(n, h1w, h0, a_dim, &need)) return kErrBadArg;
  if (!z2 || !b2 || !Wm || !h1 || !dW2 || !dWm || !dbm || !dlog_std || !workspace ||
      workspace_bytes < need) {
    set_error("mepol_head_dw2: bad arguments / workspace %zu < %zu", workspace_bytes, need);
    return kErrBadArg;
  }
  hipStream_t st = (hipStream_t)stream;
  double* coef = (double*)workspace;
  double* cpart = coef + (size_t)n * a_dim;
  double* part = cpart + (size_t)kCoefBlocks * 2 * a_dim;
  const int64_t nrc = row_chunks(n);
  const dim3 grid((unsigned)((h1w + kIB - 1) / kIB), (unsigned)((h0 + 1 + kJW - 1) / kJW),
                  (unsigned)nrc);
  hipLaunchKernelGGL(dw2_kernel, grid, dim3(256), 0, st, z2, b2, coef, Wm, h1, n, h1w, h0, a_dim,
                     part);
  MEPOL_CHECK_LAUNCH();
  const int64_t m = (int64_t)h1w * (h0 + 1) + (int64_t)a_dim * h1w + 2 * a_dim;
  hipLaunchKernelGGL(grad_reduce_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st,
                     part, (int)nrc, h1w, h0, a_dim, cpart, kCoefBlocks, dW2, db2, dWm, dbm,
                     dlog_std);
  MEPOL_CHECK_LAUNCH();
  return 0;
}
