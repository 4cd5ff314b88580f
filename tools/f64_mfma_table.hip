// f64 matrix-core issue rate on gfx950: dependency-free MFMA loops at
// several accumulator-chain counts and wave occupancies, for v_mfma_f64_16x16x4f64 and
// v_mfma_f64_4x4x4f64 (4 blocks), next to a plain v_fma_f64 loop.  Occupancy is set by dynamic
// LDS (160 KB per CU / W waves per SIMD, 256-thread blocks = one wave per SIMD each).
// Run under rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE to
// read the busy cycles per instruction next to the printed rate.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/f64_mfma_table.hip
//        -o tools/f64_mfma_table  (without the flag the f64 16x16x4 accumulators live in AGPRs
//        and every iteration copies them: 17 VALU per MFMA, the "49.6 TF/s" of round 3)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int C>
__global__ __launch_bounds__(256) void mfma16(double* out, int iters) {
  extern __shared__ double pad[];
  d4 c[C];
#pragma unroll
  for (int j = 0; j < C; ++j) c[j] = (d4){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < C; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
  }
  d4 s = c[0];
#pragma unroll
  for (int j = 1; j < C; ++j) s += c[j];
  if (threadIdx.x == 0) pad[0] = s.x;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
}

template <int C>
__global__ __launch_bounds__(256) void mfma4(double* out, int iters) {
  extern __shared__ double pad[];
  double c[C];
#pragma unroll
  for (int j = 0; j < C; ++j) c[j] = 0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < C; ++j) c[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[j], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < C; ++j) s += c[j];
  if (threadIdx.x == 0) pad[0] = s;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void fma8(double* out, int iters) {
  extern __shared__ double pad[];
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3 + j;
  const double m = 0.999999, k = 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fma(a[j], m, k);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += a[j];
  if (threadIdx.x == 0) pad[0] = s;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K>
static void time_it(const char* name, K kern, double flop_per_iter_per_wave, int W, double* out) {
  const int blocks = 256 * W * 4;  // 4 rounds of resident blocks
  const size_t lds = (160 * 1024) / W - 1024;
  const int iters = 2048;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  const double fl = (double)blocks * 4 * iters * flop_per_iter_per_wave;
  printf("%-14s waves/SIMD %d: %8.3f ms  %6.1f TF/s\n", name, W, best, fl / best / 1e9);
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 256 * 8 * 4 * sizeof(double));
  for (int W : {1, 2, 4, 8}) {
    time_it("mfma16x16 c1", mfma16<1>, 1 * 2048.0, W, out);
    time_it("mfma16x16 c2", mfma16<2>, 2 * 2048.0, W, out);
    time_it("mfma16x16 c4", mfma16<4>, 4 * 2048.0, W, out);
    time_it("mfma16x16 c8", mfma16<8>, 8 * 2048.0, W, out);
    time_it("mfma4x4 c4", mfma4<4>, 4 * 512.0, W, out);
    time_it("mfma4x4 c8", mfma4<8>, 8 * 512.0, W, out);
    time_it("v_fma_f64 x8", fma8, 8 * 64 * 2.0, W, out);
  }
  return 0;
}
