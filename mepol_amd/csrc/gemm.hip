// f64 GEMM on the CDNA4 matrix cores (v_mfma_f64_16x16x4f64) for the policy's hidden layer:
// C[n][m] = act(sum_k A[n][k] B[m][k] + bias[m]) with A [N x K] and B [M x K] row-major ("NT"),
// which is z2 = h1 W2^T of GaussianPolicy.net (src/policy.py:21-26, the 400 -> 300 Linear) and,
// with B = W2^T, dh1 = dz2 W2 of its backward.
//
// Tiling: a workgroup owns a BM x BN tile of C (WR x WC waves, each FR x FC 16x16 fragments,
// accumulators in registers), streams K through LDS in k-tiles of 16 (double-buffered, one
// barrier per tile).  Rows of both operand tiles are stored with a 144-B stride (16 + 2
// doubles): a fragment read is a ds_read_b128 whose 16 lanes of a row group hit all 64 banks
// once.  The k order inside a tile is permuted so that each lane's four k-steps are contiguous
// (lane group g = lane>>4 feeds k = 4g + s at step s for both operands), i.e. two b128 reads
// give a lane all of its fragment data for the tile.
#include "common.hpp"

namespace mepol {
namespace gemm {

constexpr int KT = 16;  // k per LDS tile
constexpr int KP = 18;  // padded LDS row (doubles)
typedef double d4 __attribute__((ext_vector_type(4)));

// XCD-aware tile order for a 1-D grid: workgroup L runs on XCD L % 8, so consecutive tiles
// (the column tiles of one row block, which share the A rows) are given to consecutive
// workgroups of the SAME XCD and meet in its L2.  A bijection on [0, ntiles).
__device__ __forceinline__ int xcd_tile(int L, int ntiles) {
  const int x = L & 7, s = L >> 3, q = ntiles >> 3, r = ntiles & 7;
  return x * q + min(x, r) + s;
}

template <int WR, int WC, int FR, int FC>
struct Cfg {
  static constexpr int kThreads = WR * WC * 64;
  static constexpr int BM = WR * FR * 16, BN = WC * FC * 16;
  static constexpr int CA = BM * (KT / 2), CB = BN * (KT / 2);  // 16-B chunks per k-tile
  static constexpr int PA = (CA + kThreads - 1) / kThreads, PB = (CB + kThreads - 1) / kThreads;
  static constexpr size_t kLds = 2ull * (BM + BN) * KP * sizeof(double);
};

template <int WR, int WC, int FR, int FC>
__global__ __launch_bounds__(WR * WC * 64) void gemm_nt_kernel(
    const double* __restrict__ A, int64_t N, int K, int64_t lda, const double* __restrict__ B,
    int M, int64_t ldb, const double* __restrict__ bias, int relu, double* __restrict__ C,
    int64_t ldc) {
  using P = Cfg<WR, WC, FR, FC>;
  constexpr int T = P::kThreads, BM = P::BM, BN = P::BN;
  extern __shared__ double lds[];
  double* sA = lds;                  // [2][BM][KP]
  double* sB = lds + 2 * BM * KP;    // [2][BN][KP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int ncb = (M + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t row0 = (int64_t)(tile / ncb) * BM;
  const int col0 = (tile % ncb) * BN;
  const int nkt = (K + KT - 1) / KT;

  double2 ra[P::PA], rb[P::PB];
  auto gload = [&](int kt) __attribute__((always_inline)) {
    const int kb = kt * KT;
#pragma unroll
    for (int p = 0; p < P::PA; ++p) {
      const int ch = tid + p * T, r = ch >> 3, k = kb + 2 * (ch & 7);
      const int64_t g = row0 + r;
      ra[p] = (ch < P::CA && g < N && k < K) ? *reinterpret_cast<const double2*>(A + g * lda + k)
                                             : double2{0.0, 0.0};
    }
#pragma unroll
    for (int p = 0; p < P::PB; ++p) {
      const int ch = tid + p * T, r = ch >> 3, k = kb + 2 * (ch & 7);
      const int c = col0 + r;
      rb[p] = (ch < P::CB && c < M && k < K) ? *reinterpret_cast<const double2*>(B + c * ldb + k)
                                             : double2{0.0, 0.0};
    }
  };
  auto lstore = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < P::PA; ++p) {
      const int ch = tid + p * T;
      if (ch < P::CA)
        *reinterpret_cast<double2*>(sA + (buf * BM + (ch >> 3)) * KP + 2 * (ch & 7)) = ra[p];
    }
#pragma unroll
    for (int p = 0; p < P::PB; ++p) {
      const int ch = tid + p * T;
      if (ch < P::CB)
        *reinterpret_cast<double2*>(sB + (buf * BN + (ch >> 3)) * KP + 2 * (ch & 7)) = rb[p];
    }
  };

  d4 acc[FR][FC];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  const int fr = lane & 15, g = lane >> 4;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) gload(kt + 1);
    double2 a[FR][2], b[FC][2];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
      const double* p = sA + (buf * BM + wr * FR * 16 + i * 16 + fr) * KP + 4 * g;
      a[i][0] = *reinterpret_cast<const double2*>(p);
      a[i][1] = *reinterpret_cast<const double2*>(p + 2);
    }
#pragma unroll
    for (int j = 0; j < FC; ++j) {
      const double* p = sB + (buf * BN + wc * FC * 16 + j * 16 + fr) * KP + 4 * g;
      b[j][0] = *reinterpret_cast<const double2*>(p);
      b[j][1] = *reinterpret_cast<const double2*>(p + 2);
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int i = 0; i < FR; ++i) {
        const double av = (s & 1) ? a[i][s >> 1].y : a[i][s >> 1].x;
#pragma unroll
        for (int j = 0; j < FC; ++j) {
          const double bv = (s & 1) ? b[j][s >> 1].y : b[j][s >> 1].x;
          acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[i][j], 0, 0, 0);
        }
      }
    }
    if (kt + 1 < nkt) lstore(buf ^ 1);
    __syncthreads();
  }

  // C/D map of the f64 16x16x4 MFMA: col = lane & 15, row = (lane >> 4) + 4 q.
#pragma unroll
  for (int j = 0; j < FC; ++j) {
    const int c = col0 + wc * FC * 16 + j * 16 + fr;
    if (c >= M) continue;
    const double bc = bias ? bias[c] : 0.0;
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + wr * FR * 16 + i * 16 + g + 4 * q;
        if (r < N) {
          double v = acc[i][j][q] + bc;
          if (relu) v = fmax(v, 0.0);
          C[r * ldc + c] = v;
        }
      }
  }
}

template <int WR, int WC, int FR, int FC>
int launch_nt(const double* A, int64_t n, int k, int64_t lda, const double* B, int m,
              int64_t ldb, const double* bias, int relu, double* C, int64_t ldc,
              hipStream_t st) {
  using P = Cfg<WR, WC, FR, FC>;
  static bool attr = false;
  if (!attr) {
    MEPOL_HIP(hipFuncSetAttribute((const void*)gemm_nt_kernel<WR, WC, FR, FC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)P::kLds));
    attr = true;
  }
  const int64_t tiles = (int64_t)((m + P::BN - 1) / P::BN) * ((n + P::BM - 1) / P::BM);
  hipLaunchKernelGGL((gemm_nt_kernel<WR, WC, FR, FC>), dim3((unsigned)tiles), dim3(P::kThreads), P::kLds, st, A,
                     n, k, lda, B, m, ldb, bias, relu, C, ldc);
  MEPOL_CHECK_LAUNCH();
  return 0;
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
  MEPOL_CHECK_LAUNCH();
  return 0;
}
}  // namespace gemm
}  // namespace mepol

using namespace mepol::gemm;

// C = act(A B^T + bias): A [n, k] (row stride lda), B [m, k] (row stride ldb), C [n, m] (row
// stride ldc), f64; k even and lda, ldb even (16-B operand loads).  `variant` picks the tiling
// (0 = default; others for tuning).
extern "C" int mepol_gemm_nt(const double* A, int64_t n, int k, int64_t lda, const double* B,
                             int m, int64_t ldb, const double* bias, int relu, double* C,
                             int64_t ldc, int variant, void* stream) {
  if (n < 0 || k <= 0 || m <= 0 || (k & 1) || (lda & 1) || (ldb & 1) || lda < k || ldb < k ||
      ldc < m || !A || !B || !C || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) {
    mepol::set_error("mepol_gemm_nt: bad arguments (k, lda, ldb even; 16-B aligned operands)");
    return mepol::kErrBadArg;
  }
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: return launch_nt<2, 2, 4, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 1: return launch_nt<4, 2, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 2: return launch_nt<2, 2, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 3: return launch_nt<4, 1, 2, 10>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 5: return launch_nt<2, 2, 4, 4>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 6: return launch_nt<2, 4, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 7: return launch_nt<4, 1, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 8: return launch_nt<2, 5, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 9: return launch_nt<8, 1, 2, 5>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    case 10: return launch_nt<4, 2, 2, 4>(A, n, k, lda, B, m, ldb, bias, relu, C, ldc, st);
    default:
      mepol::set_error("mepol_gemm_nt: unknown variant %d", variant);
      return mepol::kErrBadArg;
  }
}

// Experiment entry: DPP-broadcast VALU GEMM, same operands as mepol_gemm_nt.
extern "C" int mepol_gemm_dpp(const double* A, int64_t n, int k, int64_t lda, const double* B,
                              int m, int64_t ldb, const double* bias, int relu, double* C,
                              int64_t ldc, int variant, void* stream) {
  if (n < 0 || k <= 0 || m <= 0 || (k & 1) || (lda & 1) || (ldb & 1) || lda < k || ldb < k ||
      ldc < m || !A || !B || !C || ((uintptr_t)A & 15) || ((uintptr_t)B & 15)) {
    mepol::set_error("mepol_gemm_dpp: bad arguments (k, lda, ldb even; 16-B aligned operands)");
    return mepol::kErrBadArg;
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
    default: return mepol::kErrBadArg;
  }
}
