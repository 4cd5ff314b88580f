// Tuning experiment kept out of the product library: z2 = h1 W2^T (the policy forward's GEMM,
// K = h0 along the rows of both operands) on the f64 matrix cores with no LDS and no barrier,
// the operand shape of csrc/wgrad.hip.  A lane (m = l & 15, g = l >> 4) loads 16 B of its row
// per operand fragment, k = k0 + 2 g + {0, 1}, and the two MFMA k-steps of the stage take the
// .x / .y halves (A and B use the same k order, so the sum runs over the same products).  One
// workgroup = NW waves side by side over one 16 FO-row block, wave w owning columns
// [16 FI w, 16 FI (w + 1)).  Built by tools/variants/build_z2.sh for tools/z2_probe.py.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace z2v {
typedef double d4 __attribute__((ext_vector_type(4)));

template <int FO, int FI, int NS, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void nt_kernel(
    const double* __restrict__ A, int64_t n, int K, const double* __restrict__ B, int N,
    double* __restrict__ C) {
  constexpr int NL = FO + FI;
  const int l = threadIdx.x & 63, fr = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * 16 * FO;
  const int col0 = 16 * FI * w;
  const double* ap[FO];
  const double* bp[FI];
#pragma unroll
  for (int t = 0; t < FO; ++t) ap[t] = A + min<int64_t>(row0 + 16 * t + fr, n - 1) * K + 2 * g;
#pragma unroll
  for (int u = 0; u < FI; ++u) bp[u] = B + (int64_t)min(col0 + 16 * u + fr, N - 1) * K + 2 * g;
  d4 acc[FO][FI];
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int u = 0; u < FI; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  double2 R[NS][NL];
  const int nst = K / 8;  // probe: K % 8 == 0
  auto load = [&](double2 (&D)[NL], int st) __attribute__((always_inline)) {
    const int k = 8 * min(st, nst - 1);
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
  for (int p = 0; p < NS - 1; ++p) load(R[p], p);
  int st = 0;
#pragma nounroll
  for (; st + NS <= nst; st += NS) {
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      load(R[(p + NS - 1) % NS], st + p + NS - 1);
      mma(R[p]);
    }
  }
#pragma unroll
  for (int p = 0; p < NS; ++p)
    if (st + p < nst) {
      if (st + p + NS - 1 < nst) load(R[(p + NS - 1) % NS], st + p + NS - 1);
      mma(R[p]);
    }
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t r = row0 + 16 * t + g + 4 * q;
#pragma unroll
      for (int u = 0; u < FI; ++u) {
        const int c = col0 + 16 * u + fr;
        if (r < n && c < N) C[r * N + c] = acc[t][u][q];
      }
    }
}

template <int FO, int FI, int NS>
static void launch(const double* A, int64_t n, int K, const double* B, int N, double* C,
                   hipStream_t s) {
  constexpr int NW = (300 + 16 * FI - 1) / (16 * FI);
  const int64_t blocks = (n + 16 * FO - 1) / (16 * FO);
  hipLaunchKernelGGL((nt_kernel<FO, FI, NS, NW>), dim3((unsigned)blocks), dim3(64 * NW), 0, s,
                     A, n, K, B, N, C);
}
}  // namespace z2v

extern "C" int z2_nt(int variant, const double* A, int64_t n, int K, const double* B, int N,
                     double* C, void* stream) {
  if (K % 8 || N > 320) return -1;
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 0: z2v::launch<4, 5, 2>(A, n, K, B, N, C, s); break;
    case 1: z2v::launch<4, 4, 2>(A, n, K, B, N, C, s); break;
    case 2: z2v::launch<4, 4, 3>(A, n, K, B, N, C, s); break;
    case 3: z2v::launch<2, 5, 3>(A, n, K, B, N, C, s); break;
    case 4: z2v::launch<4, 5, 1>(A, n, K, B, N, C, s); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
