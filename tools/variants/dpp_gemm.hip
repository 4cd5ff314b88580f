// Tuning experiment kept out of the product library: the f64 GEMM of
// mepol_gemm_nt on the VALU instead of the matrix cores.  Built by tools/variants/build_dpp.sh
// into tools/variants/libdpp_gemm.so for tools/gemm_nt_probe.py (PROBE_KIND=dpp) and
// tools/vmix_probe.py.  Measured 42-44 TF/s at the C3 shapes, below the MFMA kernels, and it
// does not overlap an MFMA-bound kernel on another stream (profiles/r2/valu_mfma_overlap_probe.txt).
#include <hip/hip_runtime.h>
#include <cstdint>

namespace mepol_variants {
constexpr int kWave = 64;
// block L -> tile: consecutive tiles on one XCD (blocks are dealt round-robin over 8 XCDs)
__device__ __forceinline__ int xcd_tile(int L, int ntiles) {
  const int x = L & 7, s = L >> 3, q = ntiles >> 3, r = ntiles & 7;
  return x * q + min(x, r) + s;
}
// ---- experiment: VALU f64 GEMM with DPP row broadcast ---------------------------------------
// v_fmac_f64 issues at 68 TF/s on gfx950 against 49 TF/s for the f64 MFMA (tools/f64_rate_probe),
// so a VALU GEMM has the higher ceiling.  This form reaches 42-44 TF/s at the C3 shapes
// (tools/gemm_nt_probe.py, PROBE_KIND=dpp), below the MFMA kernel; kept for tuning.
// Lane = row; a wave owns TG groups of 16 columns.  Per k, a lane loads its A value and, per
// group, the B value of column (lane & 15); v_fmac_f64 with row_newbcast:j multiplies the
// B value of lane j of each 16-lane row (= column j of the group) into the lane's row.
template <int J>
__device__ __forceinline__ void fmac_bc(double& acc, double b, double a) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(b), "v"(a), "n"(J));
}

template <int TG, int J = 0>
__device__ __forceinline__ void fmac_group(double (&acc)[16], double b, double a) {
  if constexpr (J < 16) {
    fmac_bc<J>(acc[J], b, a);
    fmac_group<TG, J + 1>(acc, b, a);
  }
}

template <int TG, int WR, int WC>
__global__ __launch_bounds__(WR * WC * 64) void dpp_gemm_kernel(
    const double* __restrict__ A, int64_t N, int K, int64_t lda, const double* __restrict__ B,
    int M, int64_t ldb, const double* __restrict__ bias, int relu, double* __restrict__ C,
    int64_t ldc) {
  constexpr int T = WR * WC * 64, BM = 64 * WR, BN = 16 * TG * WC, KTV = 16, KPV = KTV / 2;
  constexpr int CA = BM * KPV, CB = BN * KPV, PA = (CA + T - 1) / T, PB = (CB + T - 1) / T;
  __shared__ double2 sA[2][KPV][BM];
  __shared__ double2 sB[2][KPV][BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int ncb = (M + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t row0 = (int64_t)(tile / ncb) * BM;
  const int col0 = (tile % ncb) * BN;
  const int nkt = (K + KTV - 1) / KTV;
  double acc[TG][16];
#pragma unroll
  for (int t = 0; t < TG; ++t)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[t][j] = 0.0;
  double2 ra[PA], rb[PB];
  auto gload = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int ch = tid + p * T, r = ch % BM, kp = ch / BM, k = kt * KTV + 2 * kp;
      const int64_t g = row0 + r;
      ra[p] = (ch < CA && g < N && k < K) ? *reinterpret_cast<const double2*>(A + g * lda + k)
                                          : double2{0.0, 0.0};
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int ch = tid + p * T, c = ch % BN, kp = ch / BN, k = kt * KTV + 2 * kp;
      rb[p] = (ch < CB && col0 + c < M && k < K)
                  ? *reinterpret_cast<const double2*>(B + (int64_t)(col0 + c) * ldb + k)
                  : double2{0.0, 0.0};
    }
  };
  auto lstore = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PA; ++p) {
      const int ch = tid + p * T;
      if (ch < CA) sA[buf][ch / BM][ch % BM] = ra[p];
    }
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int ch = tid + p * T;
      if (ch < CB) sB[buf][ch / BN][ch % BN] = rb[p];
    }
  };
  gload(0);
  lstore(0);
  __syncthreads();
  const int q = lane & 15;
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) gload(kt + 1);
    // register double-buffering: k-pair kp + 1's LDS reads are in flight during kp's FMAs
    double2 an = sA[buf][0][wr * 64 + lane], bn[TG];
#pragma unroll
    for (int t = 0; t < TG; ++t) bn[t] = sB[buf][0][wc * 16 * TG + 16 * t + q];
#pragma unroll
    for (int kp = 0; kp < KPV; ++kp) {
      const double2 a = an;
      double2 b[TG];
#pragma unroll
      for (int t = 0; t < TG; ++t) b[t] = bn[t];
      if (kp + 1 < KPV) {
        an = sA[buf][kp + 1][wr * 64 + lane];
#pragma unroll
        for (int t = 0; t < TG; ++t) bn[t] = sB[buf][kp + 1][wc * 16 * TG + 16 * t + q];
      }
#pragma unroll
      for (int t = 0; t < TG; ++t) fmac_group<TG>(acc[t], b[t].x, a.x);
#pragma unroll
      for (int t = 0; t < TG; ++t) fmac_group<TG>(acc[t], b[t].y, a.y);
    }
    if (kt + 1 < nkt) lstore(buf ^ 1);
    __syncthreads();
  }
  const int64_t row = row0 + wr * 64 + lane;
  if (row < N) {
#pragma unroll
    for (int t = 0; t < TG; ++t)
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int c = col0 + wc * 16 * TG + 16 * t + j;
        if (c < M) {
          double v = acc[t][j] + (bias ? bias[c] : 0.0);
          if (relu) v = fmax(v, 0.0);
          C[row * ldc + c] = v;
        }
      }
  }
}

template <int TG, int WR, int WC>
int launch_dpp(const double* A, int64_t n, int k, int64_t lda, const double* B, int m,
               int64_t ldb, const double* bias, int relu, double* C, int64_t ldc, hipStream_t st) {
  constexpr int BM = 64 * WR, BN = 16 * TG * WC;
  const int64_t tiles = (int64_t)((m + BN - 1) / BN) * ((n + BM - 1) / BM);
  hipLaunchKernelGGL((dpp_gemm_kernel<TG, WR, WC>), dim3((unsigned)tiles), dim3(WR * WC * 64), 0, st, A, n, k, lda,
                     B, m, ldb, bias, relu, C, ldc);
  if (hipGetLastError() != hipSuccess) return 1;
  return 0;
}
}  // namespace mepol_variants

using namespace mepol_variants;

// Experiment entry: DPP-broadcast VALU GEMM, same operands as mepol_gemm_nt.
extern "C" int mepol_gemm_dpp(const double* A, int64_t n, int k, int64_t lda, const double* B,
                              int m, int64_t ldb, const double* bias, int relu, double* C,
                              int64_t ldc, int variant, void* stream) {
  if (n < 0 || k <= 0 || m <= 0 || (k & 1) || (lda & 1) || (ldb & 1) || lda < k || ldb < k ||
      ldc < m || !A || !B || !C || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) {
    return 1001;
  }
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: return launch_dpp<5, 2, 2>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 1: return launch_dpp<5, 1, 4>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 2: return launch_dpp<5, 1, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 3: return launch_dpp<4, 2, 2>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 4: return launch_dpp<5, 4, 1>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 5: return launch_dpp<2, 2, 2>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 6: return launch_dpp<2, 2, 4>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 7: return launch_dpp<2, 4, 2>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 8: return launch_dpp<3, 2, 2>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 9: return launch_dpp<2, 1, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    default: return 1001;
  }
}
