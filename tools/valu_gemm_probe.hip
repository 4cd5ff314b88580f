// Probe: f64 GEMM C[M][N] = A[M][K] B[K][N] on the VALU with the broadcast operand in SGPRs.
// Lane = R rows of a 64-row tile (A read transposed, AT[K][M]: one coalesced load per row and
// k); a wave owns J output columns; B[k][j0 .. j0+J) is wave-uniform (scalar loads into SGPRs),
// so each v_fma_f64 takes one SGPR pair and needs no cross-lane traffic.
// Reports TF/s at the C3 forward shape (M = 200000, K = 400, N = 300) against the f64 MFMA
// and plain v_fma_f64 loops (tools/f64_rate_probe.hip: ~49 and ~63-68 TF/s).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_gemm_probe.hip -o tools/valu_gemm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

template <int R, int J>
__global__ __launch_bounds__(256) void valu_gemm(const double* __restrict__ AT,
                                                 const double* __restrict__ B, double* __restrict__ C,
                                                 int M, int K, int N) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int ncol = N / J;                     // column groups (N % J == 0 here)
  // one (row tile, column group) per wave; readfirstlane: the compiler then knows the B
  // pointer is wave-uniform and loads B with scalar loads
  const int wid = __builtin_amdgcn_readfirstlane((int)blockIdx.x * 4 + w);
  const long rt = wid / ncol;
  const int cg = wid % ncol;
  const long r0 = rt * 64 * R;
  if (r0 >= M) return;
  double acc[R][J];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int j = 0; j < J; ++j) acc[r][j] = 0.0;
  const double* __restrict__ Bc = B + cg * J;
  long rows[R];
#pragma unroll
  for (int r = 0; r < R; ++r) rows[r] = min(r0 + r * 64 + l, (long)M - 1);
  // A for step k + P is loaded while step k computes (P steps in flight)
  constexpr int P = 3;
  double a[P][R];
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int r = 0; r < R; ++r) a[p][r] = AT[(long)min(p, K - 1) * M + rows[r]];
  for (int k0 = 0; k0 < K; k0 += P) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int k = k0 + p;
      if (k < K) {
        const double* bk = Bc + (long)k * N;  // wave-uniform: scalar loads
        double cur[R];
#pragma unroll
        for (int r = 0; r < R; ++r) cur[r] = a[p][r];
#pragma unroll
        for (int r = 0; r < R; ++r) a[p][r] = AT[(long)min(k + P, K - 1) * M + rows[r]];
#pragma unroll
        for (int j = 0; j < J; ++j) {
          const double b = bk[j];
#pragma unroll
          for (int r = 0; r < R; ++r) acc[r][j] = fma(cur[r], b, acc[r][j]);
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const long row = r0 + r * 64 + l;
    if (row < M)
#pragma unroll
      for (int j = 0; j < J; ++j) C[row * N + cg * J + j] = acc[r][j];
  }
}

template <int R, int J>
static void run(const double* AT, const double* B, double* C, int M, int K, int N,
                const std::vector<double>& hA, const std::vector<double>& hB) {
  const long rtiles = (M + 64 * R - 1) / (64 * R);
  const long waves = rtiles * (N / J);
  const dim3 g((unsigned)((waves + 3) / 4));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((valu_gemm<R, J>), g, dim3(256), 0, 0, AT, B, C, M, K, N);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  // spot check a few entries against a host dot product
  std::vector<double> hC((size_t)M * N);
  hipMemcpy(hC.data(), C, hC.size() * 8, hipMemcpyDeviceToHost);
  double maxrel = 0;
  for (int t = 0; t < 64; ++t) {
    const long i = (long)(t * 2654435761u % M), j = t * 7 % N;
    double s = 0;
    for (int k = 0; k < K; ++k) s = fma(hA[(size_t)k * M + i], hB[(size_t)k * N + j], s);
    maxrel = fmax(maxrel, fabs(hC[i * N + j] - s) / fmax(fabs(s), 1e-300));
  }
  const double fl = 2.0 * M * (double)N * K;
  printf("R=%d J=%2d: %.3f ms  %.1f TF/s  (max rel err vs host %.1e)\n", R, J, best,
         fl / best / 1e9, maxrel);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 200000, K = argc > 2 ? atoi(argv[2]) : 400,
            N = argc > 3 ? atoi(argv[3]) : 300;
  std::vector<double> hA((size_t)K * M), hB((size_t)K * N);
  srand(1);
  for (auto& x : hA) x = rand() / (double)RAND_MAX - 0.5;
  for (auto& x : hB) x = rand() / (double)RAND_MAX - 0.5;
  double *AT, *B, *C;
  hipMalloc(&AT, hA.size() * 8);
  hipMalloc(&B, hB.size() * 8);
  hipMalloc(&C, (size_t)M * N * 8);
  hipMemcpy(AT, hA.data(), hA.size() * 8, hipMemcpyHostToDevice);
  hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice);
  printf("M=%d K=%d N=%d\n", M, K, N);
  run<1, 20>(AT, B, C, M, K, N, hA, hB);
  run<1, 30>(AT, B, C, M, K, N, hA, hB);
  run<2, 20>(AT, B, C, M, K, N, hA, hB);
  run<2, 30>(AT, B, C, M, K, N, hA, hB);
  run<4, 10>(AT, B, C, M, K, N, hA, hB);
  run<4, 15>(AT, B, C, M, K, N, hA, hB);
  run<4, 20>(AT, B, C, M, K, N, hA, hB);
  run<6, 10>(AT, B, C, M, K, N, hA, hB);
  run<8, 10>(AT, B, C, M, K, N, hA, hB);
  return 0;
}
