// Round 6 probe: the data-path floor of the k-NN select at C3 (6250 query tiles x 2 candidate
// ranges of 3125 tiles, 2 x 1-KB f16 fragments per tile, 2 MFMA 32x32x16 per wave-tile).
// Variants (no list work: each lane keeps a running min of its accumulators):
//   reg<M>   register-streamed fragments as the product kernel (3-deep ring, 4 waves per WG);
//            M bit 1 = loads, bit 2 = MFMA, bit 4 = each wave starts at a different quarter
//            of the range (no L1 sharing between the WG's waves)
//   ring<C,R,G>  fragments through an LDS ring of R tiles filled by ONE loader wave by LDS-DMA
//            and read by C consumer waves with ds_read_b128; slots are handed over by FULL /
//            FREE counters in LDS (no barrier); the loader keeps G tiles in flight
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form -o fp floor_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

using f32x16 = __attribute__((ext_vector_type(16))) float;
using f32x4 = __attribute__((ext_vector_type(4))) float;
using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
constexpr int KS = 2, NV = 2;

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__device__ __forceinline__ void make_b(f16x8 (&b)[KS], int l) {
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) b[s][j] = (_Float16)(((l * 7 + s * 3 + j) % 13) * 0.05f - 0.3f);
}

__device__ __forceinline__ float tile_min(const f32x16& acc) {
  float gm[4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
    gm[g] = fminf(fminf(acc[4 * g], acc[4 * g + 1]), fminf(acc[4 * g + 2], acc[4 * g + 3]));
  return fminf(fminf(gm[0], gm[1]), fminf(gm[2], gm[3]));
}

template <int M, int NB = 3>
__global__ __launch_bounds__(256) void reg_kernel(
    const f32x4* __restrict__ pack, int64_t tps, int64_t nct, float* __restrict__ out) {
  // M: 1 loads, 2 MFMA, 4 distinct start per wave, 8 no min tree (accumulator carried across
  // tiles: a pure MFMA chain), 16 min tree lagged by two tiles, 32 two query tiles per wave
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  f16x8 b[KS], b2[KS];
  make_b(b, l);
  make_b(b2, l + 5);
  const int64_t t0 = (int64_t)blockIdx.y * tps, t1 = std::min(nct, t0 + tps);
  const int64_t n = (M & 32) ? (t1 - t0) / 2 : t1 - t0;
  const int64_t sh = (M & 4) ? (n / 4) * w : 0;
  const f32x4* base = pack + l;
  f32x4 B[NB][NV];
  auto tile = [&](int64_t i) { int64_t j = i + sh; j -= (j >= n) ? n : 0; return t0 + j; };
  auto load = [&](f32x4 (&A)[NV], int64_t i) {
    if constexpr (M & 1) {
      const f32x4* p = base + tile(i) * 64 * NV;
#pragma unroll
      for (int v = 0; v < NV; ++v) A[v] = p[v * 64];
    }
  };
  if constexpr (!(M & 1)) {
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
      for (int v = 0; v < NV; ++v) B[bb][v] = base[(bb * NV + v) * 64];
  }
  float run = INFINITY;
  f32x16 carry = {}, carry2 = {};
  struct Acc { f32x16 a, b; };
  auto chain = [&](const f32x4 (&A)[NV]) -> Acc {
    Acc r;
    r.a = (M & 8) ? carry : f32x16{};
    r.b = (M & 8) ? carry2 : f32x16{};
    if constexpr (M & 2) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, A[s]), b[s], r.a,
                                                     0, 0, 0);
        if constexpr (M & 32)
          r.b = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, A[s]), b2[s],
                                                       r.b, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < KS; ++s) r.a[s] = A[s][0] + A[s][3];
    }
    if constexpr (M & 8) { carry = r.a; carry2 = r.b; }
    return r;
  };
  auto proc = [&](const Acc& x) {
    if constexpr (!(M & 8)) {
      run = fminf(run, tile_min(x.a));
      if constexpr (M & 32) run = fminf(run, tile_min(x.b));
    }
  };
  Acc accP = {}, accPP = {};
  int64_t i = 0;
  if (n > 0) {
#pragma unroll
    for (int bb = 0; bb < NB - 1; ++bb) load(B[bb], std::min<int64_t>(bb, n - 1));
    auto step_at = [&](int cur, bool prev) {
      load(B[(cur + NB - 1) % NB], std::min<int64_t>(i + NB - 1, n - 1));
      const Acc acc = chain(B[cur]);
      if constexpr (M & 16) {
        if (prev) proc(accPP);
        accPP = accP;
      } else {
        if (prev) proc(accP);
      }
      accP = acc;
      ++i;
    };
    step_at(0, false);
#pragma nounroll
    while (i + NB - 1 < n) {
#pragma unroll
      for (int bb = 1; bb <= NB; ++bb) step_at(bb % NB, true);
    }
#pragma unroll
    for (int bb = 1; bb < NB; ++bb)
      if (i < n) step_at(bb % NB, true);
    proc(accP);
    if constexpr (M & 16) proc(accPP);
  }
  if constexpr (M & 8) run = tile_min(carry) + tile_min(carry2);
  out[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x] = run;
}

// LDS ring: slots of one tile (NV KB); counters after the slots.
template <int C, int R, int G>
__global__ __launch_bounds__(64 * (C + 1)) void ring_kernel(const f32x4* __restrict__ pack,
                                                            int64_t tps, int64_t nct,
                                                            float* __restrict__ out) {
  __shared__ f32x4 ring[R * NV][64];
  __shared__ int full[R], freec[R];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  const int64_t t0 = (int64_t)blockIdx.y * tps, t1 = std::min(nct, t0 + tps);
  const int n = (int)(t1 - t0);
  if (threadIdx.x < R) {
    full[threadIdx.x] = 0;
    freec[threadIdx.x] = 0;
  }
  __syncthreads();
  if (w == C) {  // loader wave
    const f32x4* src = pack + t0 * 64 * NV + l;
    int pub = 0;
    for (int j = 0; j < n; ++j) {
      const int s = j % R;
      const int need = C * (j / R);
      int fc;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(fc) : "v"((unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)&freec[s]) : "memory");
      if (__builtin_amdgcn_readfirstlane(fc) < need) {
        // blocked: publish everything in flight first
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (; pub < j; ++pub)
          if (l == 0) __hip_atomic_store(&full[pub % R], pub + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        int guard = 0;
        do {
          __builtin_amdgcn_s_sleep(1);
          asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(fc) : "v"((unsigned)(uintptr_t)(__attribute__((address_space(3))) int*)&freec[s]) : "memory");
        } while (__builtin_amdgcn_readfirstlane(fc) < need && ++guard < (1 << 22));
      }
#pragma unroll
      for (int v = 0; v < NV; ++v)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(src + ((int64_t)j * NV + v) * 64),
            (__attribute__((address_space(3))) void*)&ring[s * NV + v][0], 16, 0, 0);
      if (j - pub >= G) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NV * G) : "memory");
        if (l == 0) __hip_atomic_store(&full[pub % R], pub + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ++pub;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (; pub < n; ++pub)
      if (l == 0) __hip_atomic_store(&full[pub % R], pub + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return;
  }
  f16x8 b[KS];
  make_b(b, l);
  float run = INFINITY;
  auto wait_full = [&](int j) {
    const int s = j % R;
    int guard = 0;
    while (__hip_atomic_load(&full[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != j + 1 &&
           ++guard < (1 << 22))
      __builtin_amdgcn_s_sleep(1);
    if (guard >= (1 << 22)) run = NAN;
  };
  f32x4 A[2][NV];
  f32x16 accP = {};
  if (n > 0) {
    wait_full(0);
#pragma unroll
    for (int v = 0; v < NV; ++v) A[0][v] = ring[v][l];
  }
  auto step = [&](int j, int cur, bool prev) {
    const int s = j % R;
    if (j + 1 < n) {
      wait_full(j + 1);
      const int s1 = (j + 1) % R;
#pragma unroll
      for (int v = 0; v < NV; ++v) A[cur ^ 1][v] = ring[s1 * NV + v][l];
    }
    f32x16 acc = {};
#pragma unroll
    for (int k = 0; k < KS; ++k)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, A[cur][k]), b[k], acc,
                                                   0, 0, 0);
    // slot s is in registers (the MFMAs read it): release it
    if (l == 0) __hip_atomic_fetch_add(&freec[s], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (prev) run = fminf(run, tile_min(accP));
    accP = acc;
  };
  int j = 0;
  if (n > 0) {
    step(0, 0, false);
    j = 1;
#pragma nounroll
    for (; j + 1 < n; j += 2) {
      step(j, 1, true);
      step(j + 1, 0, true);
    }
    if (j < n) step(j, 1, true);
    run = fminf(run, tile_min(accP));
  }
  out[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 64 * C + w * 64 + l] = run;
}

template <typename F>
static float time_it(F f, int reps) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  f();
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(a));
    f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = std::min(best, ms);
  }
  return best;
}

int main(int argc, char** argv) {
  const int64_t nqt = 6250, nct = 6250, split = 2, tps = (nct + split - 1) / split;
  std::vector<_Float16> h((size_t)nct * NV * 64 * 8);
  unsigned s = 12345;
  for (auto& x : h) {
    s = s * 1664525u + 1013904223u;
    x = (_Float16)((int)(s >> 9 & 0xffff) / 65536.f - 0.5f);
  }
  f32x4* pack;
  float* out;
  CHECK(hipMalloc(&pack, h.size() * 2));
  CHECK(hipMemcpy(pack, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&out, (size_t)nqt * 64 * split * 4 + (1 << 20)));
  const int reps = 5;
  const double flop = 2.0 * 32 * 32 * 32 * nqt * nct;  // issued MFMA flops
  auto rep = [&](const char* name, float ms) {
    printf("%-28s %8.3f ms  %7.1f TF/s issued\n", name, ms, flop / ms / 1e9);
    fflush(stdout);
  };
  const dim3 g4((unsigned)((nqt + 3) / 4), (unsigned)split);
  const size_t nout = (size_t)nqt * 64 * split + (1 << 18);
  std::vector<float> hout(nout);
  auto nan_check = [&](const char* name) {
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hout.data(), out, nout * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (float x : hout) bad += x != x;
    if (bad) printf("  %s: %zu NaN outputs (spin guard hit)\n", name, bad);
  };
  // lds = dynamic LDS per WG: 52000 B holds the product's occupancy (3 WGs of 4 waves per CU)
#define REG(M, LDS) rep("reg<" #M "> lds " #LDS, time_it([&] { hipLaunchKernelGGL(reg_kernel<M>, g4, dim3(256), LDS, 0, pack, tps, nct, out); }, reps))
  REG(3, 52000);
  REG(1, 52000);
  REG(2, 52000);
  REG(2, 0);
  REG(10, 52000);
  REG(18, 52000);
  REG(19, 52000);
  REG(19, 0);
  REG(34, 52000);
  REG(35, 52000);
  REG(51, 52000);
  REG(42, 52000);
#define RING(C, R, G)                                                                         \
  rep("ring<" #C "," #R "," #G ">",                                                           \
      time_it([&] {                                                                           \
        hipLaunchKernelGGL((ring_kernel<C, R, G>), dim3((unsigned)((nqt + C - 1) / C), split), \
                           dim3(64 * (C + 1)), 0, 0, pack, tps, nct, out);                     \
      }, reps));                                                                              \
  nan_check("ring<" #C "," #R "," #G ">")
  RING(11, 32, 14);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  return 0;
}
