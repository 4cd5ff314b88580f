// DROPPED (round 6, measured slower): mepol_dh1_layer1_backward_masked with its main loop in
// the no-LDS shape of z2_head_kernel / wgrad_kernel.  Correct (max |err| vs
// torch f64 4.4e-11 on |dW| ~ 2e3, as the LDS form), but at C3 (tools/dh1_ab.py): 1261 us alone
// and 2182 us beside dW2 at one wave per SIMD (256 VGPRs + 186 AGPRs), 1469 / 2348 us at two
// (275 spilled VGPRs: the 64 x 80 accumulator tile leaves no room for the epilogue), against
// 1148 / 2041 us for the LDS form (profiles/r6/f64/dh1_nolds_dropped.txt).  It was dispatched
// from dh1_layer1_backward<MASK=true> with the LDS form's grid and partials.  Not built.
#include "../../mepol_amd/csrc/common.hpp"
// Round 6: the same dh1 GEMM + layer-1 backward with its main loop in the no-LDS shape of
// z2_head_kernel / wgrad_kernel: 4 waves x (64 rows x 80 columns) per
// 256 x 80 tile, both operands (dz2 rows, W2^T rows) read straight from L2 into the MFMA
// fragments -- a lane takes 16 B of its row per fragment, k = 8 st + 2 g + {0, 1} -- with no LDS
// staging and no barrier in the K loop (the LDS form's A tile was used by one wave only, and
// its per-k-tile barriers held MFMA busy at ~0.64 against ~0.72 for the no-LDS kernels,
// profiles/r6/ck2/mlp_counters.txt).  Epilogue: the masked product dz1^T [x | 1] per column
// fragment on the matrix cores as before, one row fragment at a time (x and mask words from
// L1), reduced over the 4 waves through LDS into the same row-block partials.
namespace l1n {
constexpr int NW = 4, FO = 4, FI = 5, NS = 2, NL = FO + FI;
constexpr int BM = NW * 16 * FO, BN = 16 * FI;  // 256 x 80, the LDS form's tile
static_assert(BM == l1b::P::BM && BN == l1b::P::BN, "same tiles and partials as dh1_layer1_bwd");
}  // namespace l1n

template <int NH>
__global__ __launch_bounds__(64 * l1n::NW) __attribute__((amdgpu_waves_per_eu(MEPOL_DH1_OCC))) void
dh1_nolds_kernel(const double* __restrict__ dz2, int64_t N, int K, const double* __restrict__ W2t,
                 int M, const uint16_t* __restrict__ hm, const double* __restrict__ x, int F,
                 double* __restrict__ part) {
  using namespace l1n;
  constexpr int NE = NH * 4 * 64;
  __shared__ double red[NW * NE];
  const int tid = threadIdx.x, l = tid & 63, fr = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = (M + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int rb = tile / ncb;
  const int64_t row0 = (int64_t)rb * BM, wr0 = row0 + 64 * w;
  const int col0 = (tile % ncb) * BN;
  const double* ap[FO];
  const double* bp[FI];
#pragma unroll
  for (int t = 0; t < FO; ++t) ap[t] = dz2 + min<int64_t>(wr0 + 16 * t + fr, N - 1) * K + 2 * g;
#pragma unroll
  for (int u = 0; u < FI; ++u) bp[u] = W2t + (int64_t)min(col0 + 16 * u + fr, M - 1) * K + 2 * g;
  d4 acc[FO][FI];
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int u = 0; u < FI; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  // stage st reads k = 8 st + 2 g (+1); K is even, so a pair is whole or past the end: the
  // address is clamped to the last pair and the tail stage's pairs past K are zeroed at use
  const int nst = (K + 7) / 8, nfull = K / 8;
  double2 R[NS][NL];
  auto load = [&](double2 (&D)[NL], int st) __attribute__((always_inline)) {
    const int k = min(8 * st, K - 2 - 2 * g);
#pragma unroll
    for (int t = 0; t < FO; ++t) D[t] = *reinterpret_cast<const double2*>(ap[t] + k);
#pragma unroll
    for (int u = 0; u < FI; ++u) D[FO + u] = *reinterpret_cast<const double2*>(bp[u] + k);
  };
  auto mma = [&](const double2 (&D)[NL]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < FO; ++t)
#pragma unroll
      for (int u = 0; u < FI; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(D[t].x, D[FO + u].x, acc[t][u], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < FO; ++t)
#pragma unroll
      for (int u = 0; u < FI; ++u)
        acc[t][u] = __builtin_amdgcn_mfma_f64_16x16x4f64(D[t].y, D[FO + u].y, acc[t][u], 0, 0, 0);
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p) load(R[p], min(p, nst - 1));
  int st = 0;
#pragma nounroll
  for (; st + NS <= nfull; st += NS) {
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      load(R[(p + NS - 1) % NS], min(st + p + NS - 1, nst - 1));
      mma(R[p]);
    }
  }
#pragma unroll
  for (int p = 0; p < NS; ++p) {
    if (st + p < nst) {  // uniform
      if (st + p + NS - 1 < nst) load(R[(p + NS - 1) % NS], st + p + NS - 1);
      if (st + p >= nfull && 8 * (st + p) + 2 * g >= K) {  // the tail stage's missing pairs
#pragma unroll
        for (int v = 0; v < NL; ++v) R[p][v] = double2{0.0, 0.0};
      }
      mma(R[p]);
    }
  }

  // ---- epilogue: acc[t][u][q] = dh1[row wr0 + 16 t + g + 4 q][col col0 + 16 u + fr] ----------
  // 1. dz1 = dh1 * relu'(h1) in place (the mask words of one row fragment at a time)
  const int mw = (M + 15) / 16;
#pragma unroll
  for (int i = 0; i < FO; ++i) {
    uint32_t hv[4][FI];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t r = min<int64_t>(wr0 + 16 * i + 4 * q + g, N - 1);
#pragma unroll
      for (int j = 0; j < FI; ++j) hv[q][j] = hm[r * mw + min((col0 >> 4) + j, mw - 1)];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool rin = wr0 + 16 * i + 4 * q + g < N;
#pragma unroll
      for (int j = 0; j < FI; ++j) {
        const bool on = rin && col0 + 16 * j + fr < M && ((hv[q][j] >> fr) & 1u) != 0;
        acc[i][j][q] = on ? acc[i][j][q] : 0.0;
      }
    }
  }
  // 2. per column fragment j: dz1^T [x | 1] over the wave's 64 rows on the matrix cores
  //    (k-step (i, q): A[m = fr][k = g] = dz1 at (row 16 i + 4 q + g, col fr of fragment j),
  //    B[k = g][n = fr] = [x | 1] at (that row, feature 16 h + fr)), then the sum of the 4 waves
#pragma unroll
  for (int j = 0; j < FI; ++j) {
    // x is re-read for every j (L1): an opaque base keeps the compiler from hoisting all of
    // it out of the j loop, next to the 160 accumulator registers
    const double* xj = x;
    asm volatile("" : "+s"(xj));
    d4 dacc[NH];
#pragma unroll
    for (int h = 0; h < NH; ++h) dacc[h] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 0; i < FO; ++i) {
      double xb[4][NH];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = min<int64_t>(wr0 + 16 * i + 4 * q + g, N - 1);
#pragma unroll
        for (int h = 0; h < NH; ++h) xb[q][h] = xj[r * F + min(16 * h + fr, F - 1)];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool rin = wr0 + 16 * i + 4 * q + g < N;
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          // arithmetic, not a select (the clamped x value is a finite coordinate: x * 0 = 0)
          const int f = 16 * h + fr;
          const double keep = (rin && f < F) ? 1.0 : 0.0, one = (rin && f == F) ? 1.0 : 0.0;
          dacc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[i][j][q], fma(xb[q][h], keep, one),
                                                         dacc[h], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[((w * NH + h) * 4 + q) * 64 + l] = dacc[h][q];
    __syncthreads();
    for (int e = tid; e < NE; e += 64 * NW) {
      double sum = red[e];
#pragma unroll
      for (int v = 1; v < NW; ++v) sum += red[v * NE + e];
      const int ll = e & 63, q = (e >> 6) & 3, h = e >> 8;
      const int cc = col0 + j * 16 + (ll >> 4) + 4 * q, f = 16 * h + (ll & 15);
      if (cc < M && f <= F) part[((int64_t)rb * M + cc) * (F + 1) + f] = sum;
    }
    __syncthreads();
  }
}

