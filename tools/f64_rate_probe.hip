// Measures the f64 MFMA (v_mfma_f64_16x16x4f64) and VALU v_fma_f64 issue rates on the device.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void mfma_loop(double* out, int iters) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
}

__global__ __launch_bounds__(256) void mfma_loop8(double* out, int iters) {
  d4 c[8];
  for (int j = 0; j < 8; ++j) c[j] = (d4){0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
  }
  d4 s = c[0];
  for (int j = 1; j < 8; ++j) s += c[j];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
}

__global__ __launch_bounds__(256) void fma_loop(double* out, int iters) {
  double a[8];
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3 + j;
  const double m = 0.999999, k = 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fma(a[j], m, k);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += a[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int J>
__device__ __forceinline__ void fmac_bc(double& acc, double b, double a) {
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(acc)
               : "v"(b), "v"(a), "n"(J));
}

// v_fmac_f64 with a DPP row broadcast of src0 (the VALU GEMM's inner instruction).
__global__ __launch_bounds__(256) void dpp_loop(double* out, int iters) {
  double acc[16];
  for (int j = 0; j < 16; ++j) acc[j] = 0.0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int i = 0; i < iters; ++i) {
    fmac_bc<0>(acc[0], b, a); fmac_bc<1>(acc[1], b, a); fmac_bc<2>(acc[2], b, a);
    fmac_bc<3>(acc[3], b, a); fmac_bc<4>(acc[4], b, a); fmac_bc<5>(acc[5], b, a);
    fmac_bc<6>(acc[6], b, a); fmac_bc<7>(acc[7], b, a); fmac_bc<8>(acc[8], b, a);
    fmac_bc<9>(acc[9], b, a); fmac_bc<10>(acc[10], b, a); fmac_bc<11>(acc[11], b, a);
    fmac_bc<12>(acc[12], b, a); fmac_bc<13>(acc[13], b, a); fmac_bc<14>(acc[14], b, a);
    fmac_bc<15>(acc[15], b, a);
  }
  double s = 0;
  for (int j = 0; j < 16; ++j) s += acc[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Interleaved: 4 f64 MFMAs + 8*R independent v_fma_f64 per iteration (co-issue check).
template <int R>
__global__ __launch_bounds__(256) void mixed_loop(double* out, int iters) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  double v[8];
  for (int j = 0; j < 8; ++j) v[j] = threadIdx.x * 1e-3 + j;
  const double m = 0.999999, k = 1e-9;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 0; j < 2; ++j) v[j] = fma(v[j], m, k);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 2; j < 4; ++j) v[j] = fma(v[j], m, k);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 4; j < 6; ++j) v[j] = fma(v[j], m, k);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int j = 6; j < 8; ++j) v[j] = fma(v[j], m, k);
  }
  d4 s = c0 + c1 + c2 + c3;
  double t = 0;
  for (int j = 0; j < 8; ++j) t += v[j];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w + t;
}

int main() {
  double* out;
  hipMalloc(&out, 256 * 8192 * sizeof(double));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 4096;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)blocks * 4 * iters * 4 * 2048.0;
    printf("mfma_f64_16x16x4: %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mfma_loop8, dim3(blocks), dim3(256), 0, 0, out, iters / 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("mfma_f64_16x16x4 (8 chains): %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(fma_loop, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    fl = (double)blocks * 256 * iters * 8 * 2.0;
    printf("v_fma_f64: %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(dpp_loop, dim3(blocks), dim3(256), 0, 0, out, iters / 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("v_fmac_f64_dpp row_newbcast: %.3f ms  %.1f TF/s\n", ms, fl / ms / 1e9);
  }
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0);
    hipLaunchKernelGGL(mixed_loop<1>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double mf = (double)blocks * 4 * iters * 4 * 2048.0, vf = (double)blocks * 256 * iters * 8 * 2.0;
    printf("mixed R=1: %.3f ms  mfma %.1f + valu %.1f TF/s\n", ms, mf / ms / 1e9, vf / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(mixed_loop<4>, dim3(blocks), dim3(256), 0, 0, out, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    vf *= 4;
    printf("mixed R=4: %.3f ms  mfma %.1f + valu %.1f TF/s\n", ms, mf / ms / 1e9, vf / ms / 1e9);
  }
  return 0;
}
