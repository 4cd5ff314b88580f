// f64 GEMM on the CDNA4 matrix cores (v_mfma_f64_16x16x4f64) for the policy's hidden layer:
// C[n][m] = act(sum_k A[n][k] B[m][k] + bias[m]) with A [N x K] and B [M x K] row-major ("NT"),
// which is z2 = h1 W2^T of GaussianPolicy.net (src/policy.py:21-26, the 400 -> 300 Linear) and,
// with B = W2^T, dh1 = dz2 W2 of its backward.
//
// Tiling: a workgroup owns a BM x BN tile of C (WR x WC waves, each FR x FC 16x16 fragments,
// accumulators in registers), streams K through LDS in k-tiles of 16 (double-buffered, one
// barrier per tile).  The k order inside a tile is permuted so that each lane's four k-steps
// are contiguous (lane group g = lane>>4 feeds k = 4g + s at step s for both operands), i.e.
// two b128 reads give a lane all of its fragment data for the tile.  Rows of both operand
// tiles are 128 B (two to a 256-B bank row) with the 16-B slots XOR-swizzled per row
// (lds_slot): a ds_read_b128 is serviced in the lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31} (+32), i.e. rows fr 0-3, 12-15 of one k-slot with rows 4-11 of the next
// one, and the swizzle puts each group's 16 reads on 16 distinct slots (the round-5 144-B
// padded stride left two of them 2-way: SQ_LDS_BANK_CONFLICT 3.3e7 per C3 dh1 call); the
// stores (8-lane groups, one row) stay conflict-free.
#include "common.hpp"

#include <type_traits>

namespace mepol {
namespace gemm {

constexpr int KT = 16;  // k per LDS tile
constexpr int KP = 16;  // LDS row (doubles), swizzled by lds_slot

// physical 16-B slot of logical slot c (k = 2c, 2c + 1 of the tile) in LDS row r: c ^ h(r) with
// h(r) in {0, 1, 4, 5} from bits 1 and 3 of r.  Read group {rows 0-3, 12-15 at slot j, rows
// 4-11 at j + 2}: h over rows {0, 2, 12, 14} (and the odd ones) is {0, 1, 4, 5}, over rows
// {4, 6, 8, 10} the same set, so j ^ h and (j + 2) ^ h never meet (bit 1 differs).
__device__ __forceinline__ int lds_slot(int r, int c) {
  return c ^ (((r >> 1) & 1) | (((r >> 3) & 1) << 2));
}
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

// The main loop shared by the kernels below: acc[i][j] += A[rows of fragment i] B[cols of
// fragment j]^T over all of K for the workgroup tile (row0, col0).  Operand loads read clamped
// (always valid) addresses; out-of-range values are zeroed when the registers are written to
// LDS, after the MFMA block, so no select waits on a load right after issuing it.
// DEEP: two register sets, the global loads of tile t + 2 issued while tile t is computed (the
// store of tile t + 1 then waits on loads a whole tile older); 24 more VGPRs.
// BT: B given as [K][M] row-major (ldb = its row stride, M even, 16-B aligned rows): a lane loads
// B[k][m, m + 1] (consecutive lanes consecutive m: coalesced) and writes the pair into LDS rows
// m and m + 1 of the [BN][KT] image (two 8-B stores).  Lets dh1 = dz2 W2 read the Linear weight
// as stored instead of a per-step W2^T copy.
template <int WR, int WC, int FR, int FC, bool DEEP = false, bool BT = false>
__device__ __forceinline__ void gemm_mainloop(const double* __restrict__ A, int64_t N, int K,
                                              int64_t lda, const double* __restrict__ B, int M,
                                              int64_t ldb, int64_t row0, int col0, double* lds,
                                              d4 (&acc)[FR][FC]) {
  using P = Cfg<WR, WC, FR, FC>;
  constexpr int T = P::kThreads, BM = P::BM, BN = P::BN;
  double* sA = lds;                  // [2][BM][KP]
  double* sB = lds + 2 * BM * KP;    // [2][BN][KP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int nkt = (K + KT - 1) / KT;
  const int k2 = K - 2;  // last 16-B aligned pair start (K even)

  using RA = double2[P::PA];
  using RB = double2[P::PB];
  auto gload = [&](int kt, RA& ra, RB& rb) __attribute__((always_inline)) {
    const int kb = kt * KT;
#pragma unroll
    for (int p = 0; p < P::PA; ++p) {
      const int ch = min(tid + p * T, P::CA - 1), r = ch >> 3, k = kb + 2 * (ch & 7);
      ra[p] = *reinterpret_cast<const double2*>(A + min<int64_t>(row0 + r, N - 1) * lda +
                                                min(k, k2));
    }
#pragma unroll
    for (int p = 0; p < P::PB; ++p) {
      const int ch = min(tid + p * T, P::CB - 1);
      if constexpr (BT) {
        const int kl = ch / (BN / 2), m = 2 * (ch % (BN / 2));
        rb[p] = *reinterpret_cast<const double2*>(B + (int64_t)min(kb + kl, K - 1) * ldb +
                                                  min(col0 + m, M - 2));
      } else {
        const int r = ch >> 3, k = kb + 2 * (ch & 7);
        rb[p] = *reinterpret_cast<const double2*>(B + (int64_t)min(col0 + r, M - 1) * ldb +
                                                  min(k, k2));
      }
    }
  };
  auto lstore = [&](int kt, int buf, const RA& ra, const RB& rb) __attribute__((always_inline)) {
    const int kb = kt * KT;
#pragma unroll
    for (int p = 0; p < P::PA; ++p) {
      const int ch = tid + p * T, r = ch >> 3, k = kb + 2 * (ch & 7);
      if (ch < P::CA) {
        const bool ok = row0 + r < N && k < K;
        *reinterpret_cast<double2*>(sA + (buf * BM + r) * KP + 2 * lds_slot(r, ch & 7)) =
            ok ? ra[p] : double2{0.0, 0.0};
      }
    }
#pragma unroll
    for (int p = 0; p < P::PB; ++p) {
      const int ch = tid + p * T;
      if (ch < P::CB) {
        if constexpr (BT) {
          const int kl = ch / (BN / 2), m = 2 * (ch % (BN / 2));
          const bool ok = col0 + m < M && kb + kl < K;  // M even: m + 1 < M with m
          const int off = 2 * lds_slot(m, kl >> 1) + (kl & 1);  // rows m, m + 1: same swizzle
          const int off1 = 2 * lds_slot(m + 1, kl >> 1) + (kl & 1);
          sB[(buf * BN + m) * KP + off] = ok ? rb[p].x : 0.0;
          sB[(buf * BN + m + 1) * KP + off1] = ok ? rb[p].y : 0.0;
        } else {
          const int r = ch >> 3, k = kb + 2 * (ch & 7);
          const bool ok = col0 + r < M && k < K;
          *reinterpret_cast<double2*>(sB + (buf * BN + r) * KP + 2 * lds_slot(r, ch & 7)) =
              ok ? rb[p] : double2{0.0, 0.0};
        }
      }
    }
  };

#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  const int fr = lane & 15, g = lane >> 4;
  // a lane's two slots in its fragment rows (every fragment row is fr mod 16: same swizzle)
  const int sl0 = 2 * lds_slot(fr, 2 * g), sl1 = 2 * lds_slot(fr, 2 * g + 1);
  auto compute = [&](int buf) __attribute__((always_inline)) {
    double2 a[FR][2], b[FC][2];
#pragma unroll
    for (int i = 0; i < FR; ++i) {
      const double* p = sA + (buf * BM + wr * FR * 16 + i * 16 + fr) * KP;
      a[i][0] = *reinterpret_cast<const double2*>(p + sl0);
      a[i][1] = *reinterpret_cast<const double2*>(p + sl1);
    }
#pragma unroll
    for (int j = 0; j < FC; ++j) {
      const double* p = sB + (buf * BN + wc * FC * 16 + j * 16 + fr) * KP;
      b[j][0] = *reinterpret_cast<const double2*>(p + sl0);
      b[j][1] = *reinterpret_cast<const double2*>(p + sl1);
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
  };

  RA ra0, ra1;
  RB rb0, rb1;
  gload(0, ra0, rb0);
  lstore(0, 0, ra0, rb0);
  if constexpr (DEEP) {
    if (nkt > 1) gload(1, ra1, rb1);
    __syncthreads();
    int kt = 0;
    for (; kt + 1 < nkt; kt += 2) {  // tile kt in buffer 0, kt + 1 in buffer 1
      if (kt + 2 < nkt) gload(kt + 2, ra0, rb0);
      compute(0);
      lstore(kt + 1, 1, ra1, rb1);
      __syncthreads();
      if (kt + 3 < nkt) gload(kt + 3, ra1, rb1);
      compute(1);
      if (kt + 2 < nkt) lstore(kt + 2, 0, ra0, rb0);
      __syncthreads();
    }
    if (kt < nkt) {
      compute(0);
      __syncthreads();
    }
  } else {
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nkt) gload(kt + 1, ra0, rb0);
      compute(buf);
      if (kt + 1 < nkt) lstore(kt + 1, buf ^ 1, ra0, rb0);
      __syncthreads();
    }
  }
}

template <int WR, int WC, int FR, int FC>
__global__ __launch_bounds__(WR * WC * 64) void gemm_nt_kernel(
    const double* __restrict__ A, int64_t N, int K, int64_t lda, const double* __restrict__ B,
    int M, int64_t ldb, const double* __restrict__ bias, int relu, double* __restrict__ C,
    int64_t ldc) {
  using P = Cfg<WR, WC, FR, FC>;
  constexpr int BM = P::BM, BN = P::BN;
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int fr = lane & 15, g = lane >> 4;
  const int ncb = (M + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int64_t row0 = (int64_t)(tile / ncb) * BM;
  const int col0 = (tile % ncb) * BN;
  d4 acc[FR][FC];
  gemm_mainloop<WR, WC, FR, FC>(A, N, K, lda, B, M, ldb, row0, col0, lds, acc);

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

// ---- dh1 GEMM + first-layer backward (GaussianPolicy.net[0], src/policy.py:21-26) ------------
// dh1 = dz2 W2 is never written: the epilogue masks it with relu'(h1) (h1 > 0, read from the
// forward's h1) and reduces dz1^T [x | 1] over the tile's rows on the matrix cores, i.e. the
// tile's contribution to dW1 (and db1 in column F).  The MFMA accumulator of dh1 already is
// the A operand of that product (its k index = row); x comes from HBM as the B operand.
// Row-block partials part[rb][c][F + 1] are summed in a fixed order by layer1_reduce_kernel.
// Tiling: 8 waves x (32 rows x 80 cols), 256 x 80 tile: 5 column tiles for h0 = 400.
namespace l1b {
constexpr int WR = 8, WC = 1, FR = 2, FC = 5;
using P = Cfg<WR, WC, FR, FC>;
}  // namespace l1b

// MASK: relu'(h1) comes as the forward's bit mask (uint16 word kt of row r holds
// h1[r][16 kt + b] > 0 in bit b, mepol_policy_forward_masked) instead of the f64 h1 values:
// 2 B per 16 columns instead of 128 B, which the epilogue waited for with the MFMAs idle
// (one workgroup per CU).  The same bits either way.
// BT: W2t is the Linear weight W2 as stored, [K][M] (gemm_mainloop's BT)
template <int NH, bool MASK, bool BT>  // NH = ceil((F + 1) / 16) column groups of [x | 1]
__global__ __launch_bounds__(l1b::P::kThreads) void dh1_layer1_bwd_kernel(
    const double* __restrict__ dz2, int64_t N, int K, const double* __restrict__ W2t, int M,
    const void* __restrict__ h1v, const double* __restrict__ x, int F,
    double* __restrict__ part) {
  using namespace l1b;
  constexpr int BM = P::BM, BN = P::BN, T = P::kThreads;
  extern __shared__ double lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, g = lane >> 4;
  const int ncb = (M + BN - 1) / BN;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int rb = tile / ncb;
  const int64_t row0 = (int64_t)rb * BM;
  const int col0 = (tile % ncb) * BN;
  d4 acc[FR][FC];
  gemm_mainloop<WR, WC, FR, FC, true, BT>(dz2, N, K, K, W2t, M, BT ? M : K, row0, col0, lds,
                                         acc);

  // Every epilogue operand in ONE batch of unconditional loads (clamped addresses) before the
  // first use: the ReLU mask of h1 at the wave's accumulator elements and the [x | 1] operands.
  // Loaded where they were used, the h1 loads waited out their HBM latency in FC batches
  // (0.40 of the kernel's 1.23 ms went to this epilogue, profiles/r5/f64/).
  // B operands [x | 1] for k-step (i, q): lane (fr, g) holds x[row(i, q, g)][16 h + fr]
  double xb[FR][4][NH];
  using HT = typename std::conditional<MASK, uint32_t, double>::type;
  HT hv[FC][FR][4];
  const double* h1 = static_cast<const double*>(h1v);
  const uint16_t* hm = static_cast<const uint16_t*>(h1v);
  const int mw = (M + 15) / 16;
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // accumulator element (row g + 4 q of fragment i, col fr) is A[m = fr][k = g] of
      // k-step (i, q): rows 16 i + 4 q + g
      const int64_t r = row0 + wave * FR * 16 + i * 16 + 4 * q + g;
      const double* xr = x + min<int64_t>(r, N - 1) * F;
#pragma unroll
      for (int h = 0; h < NH; ++h) xb[i][q][h] = xr[min(16 * h + fr, F - 1)];
      if constexpr (MASK) {
        const uint16_t* mr = hm + min<int64_t>(r, N - 1) * mw;
#pragma unroll
        for (int j = 0; j < FC; ++j) hv[j][i][q] = mr[min((col0 >> 4) + j, mw - 1)];
      } else {
        const double* hr = h1 + min<int64_t>(r, N - 1) * M;
#pragma unroll
        for (int j = 0; j < FC; ++j) hv[j][i][q] = hr[min(col0 + j * 16 + fr, M - 1)];
      }
    }
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool rin = row0 + wave * FR * 16 + i * 16 + 4 * q + g < N;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        // arithmetic, not a select: a select lets hipcc sink the load into a branch and wait
        // for it there (the clamped x value is a finite state coordinate: x * 0 = 0)
        const int f = 16 * h + fr;
        const double keep = (rin && f < F) ? 1.0 : 0.0, one = (rin && f == F) ? 1.0 : 0.0;
        xb[i][q][h] = fma(xb[i][q][h], keep, one);
      }
    }
  // The wave partials of JB column fragments per LDS round (2 when they fit beside each other:
  // 6 workgroup barriers instead of 10 for FC = 5); the per-element sum over the WR waves keeps
  // its order.  The main loop's last barrier retired its LDS reads.
  constexpr int NE = NH * 4 * 64;
  constexpr int JB = 2 * WR * NE * sizeof(double) <= P::kLds ? 2 : 1;
  double* red = lds;  // [JB][WR][NH][4][64]
#pragma unroll
  for (int j0 = 0; j0 < FC; j0 += JB) {
#pragma unroll
    for (int jj = 0; jj < JB; ++jj) {
      const int j = j0 + jj;
      if (j < FC) {
        const int c = col0 + j * 16 + fr;
        d4 dacc[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) dacc[h] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < FR; ++i)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            bool on;
            if constexpr (MASK)
              on = ((hv[j][i][q] >> fr) & 1u) != 0;
            else
              on = hv[j][i][q] > 0.0;
            const double dz = (on && c < M) ? acc[i][j][q] : 0.0;
#pragma unroll
            for (int h = 0; h < NH; ++h)
              dacc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(dz, xb[i][q][h], dacc[h], 0, 0, 0);
          }
        // dacc[h][r'] = sum over the wave's rows of dz1[.][col0 + 16 j + g + 4 r'] *
        // [x|1][16 h + fr]
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int q = 0; q < 4; ++q)
            red[(jj * WR + wave) * NE + (h * 4 + q) * 64 + lane] = dacc[h][q];
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < JB * NE; e += T) {
      const int jj = e / NE, ee = e - jj * NE, j = j0 + jj;
      if (j < FC) {
        double s = red[jj * WR * NE + ee];
#pragma unroll
        for (int w = 1; w < WR; ++w) s += red[(jj * WR + w) * NE + ee];
        const int l = ee & 63, q = (ee >> 6) & 3, h = ee >> 8;
        const int cc = col0 + j * 16 + (l >> 4) + 4 * q, f = 16 * h + (l & 15);
        if (cc < M && f <= F) part[((int64_t)rb * M + cc) * (F + 1) + f] = s;
      }
    }
    __syncthreads();
  }
}

// dW[c][f] = sum_b part[b][c][f], db[c] = sum_b part[b][c][F] in two fixed-order stages: stage 1
// sums row-block group g (kGroups of them, strided rows) for 64 elements per block; stage 2 sums
// the groups in order.  (One block column per 64 elements with all row blocks serial was
// latency-bound at 79 us for 782 x 12000 partials.)
constexpr int kGroups = 16;

__global__ __launch_bounds__(256) void layer1_reduce_kernel(const double* __restrict__ part,
                                                            int nb, int M, int F,
                                                            double* __restrict__ grp) {
  __shared__ double sh[4][64];
  const int64_t m = (int64_t)M * (F + 1);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + l;
  const int gi = blockIdx.y;
  double s = 0.0;
  if (e < m)
    for (int b = gi + kGroups * w; b < nb; b += 4 * kGroups) s += part[(int64_t)b * m + e];
  sh[w][l] = s;
  __syncthreads();
  if (w == 0 && e < m) grp[(int64_t)gi * m + e] = sh[0][l] + sh[1][l] + sh[2][l] + sh[3][l];
}

__global__ __launch_bounds__(256) void layer1_reduce2_kernel(const double* __restrict__ grp,
                                                             int M, int F,
                                                             double* __restrict__ dW,
                                                             double* __restrict__ db) {
  const int64_t m = (int64_t)M * (F + 1);
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= m) return;
  double t = 0.0;
#pragma unroll
  for (int g = 0; g < kGroups; ++g) t += grp[(int64_t)g * m + e];
  const int c = (int)(e / (F + 1)), f = (int)(e % (F + 1));
  if (f < F)
    dW[(int64_t)c * F + f] = t;
  else if (db)
    db[c] = t;
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


// dW1 [m, F], db1 [m] (nullable) of h1 = relu(x W1^T + b1) given dz2 [n, k] and W2t = W2^T
// [m, k] (dh1 = dz2 W2 = dz2 W2t^T, not materialised), the forward's h1 [n, m] and x [n, F].
extern "C" int mepol_dh1_layer1_workspace_size(int64_t n, int m, int in_features,
                                               size_t* bytes) {
  using namespace mepol::gemm::l1b;
  if (!bytes) return mepol::kErrBadArg;
  *bytes = ((size_t)((n + P::BM - 1) / P::BM) + mepol::gemm::kGroups) * m * (in_features + 1) *
           sizeof(double);
  return 0;
}

template <bool MASK, bool BT = false>
static int dh1_layer1_backward(const double* dz2, int64_t n, int k, const double* W2t, int m,
                               const void* h1, const double* x, int in_features, double* dW1,
                               double* db1, void* workspace, size_t workspace_bytes,
                               void* stream) {
  using namespace mepol::gemm::l1b;
  using mepol::gemm::dh1_layer1_bwd_kernel;
  const int F = in_features;
  if (n <= 0 || k <= 0 || (k & 1) || m <= 0 || F <= 0 || F > 63 || !dz2 || !W2t || !h1 || !x ||
      !dW1 || !workspace || ((uintptr_t)dz2 & 15) || ((uintptr_t)W2t & 15) || (BT && (m & 1))) {
    mepol::set_error("mepol_dh1_layer1_backward: bad arguments (k even, in_features <= 63, "
                     "16-B aligned dz2 / W2t)");
    return mepol::kErrBadArg;
  }
  const int nrb = (int)((n + P::BM - 1) / P::BM);
  const size_t need = ((size_t)nrb + mepol::gemm::kGroups) * m * (F + 1) * sizeof(double);
  if (workspace_bytes < need) {
    mepol::set_error("mepol_dh1_layer1_backward: workspace %zu < %zu", workspace_bytes, need);
    return mepol::kErrWorkspace;
  }
  hipStream_t st = (hipStream_t)stream;
  const int ncb = (m + P::BN - 1) / P::BN;
  const unsigned tiles = (unsigned)((int64_t)nrb * ncb);
  double* part = (double*)workspace;
  const int nh = (F + 1 + 15) / 16;
#define MEPOL_L1B(NHV)                                                                         \
  do {                                                                                         \
    static bool attr = false;                                                                  \
    if (!attr) {                                                                               \
      MEPOL_HIP(hipFuncSetAttribute((const void*)dh1_layer1_bwd_kernel<NHV, MASK, BT>,         \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)P::kLds)); \
      attr = true;                                                                             \
    }                                                                                          \
    hipLaunchKernelGGL((dh1_layer1_bwd_kernel<NHV, MASK, BT>), dim3(tiles), dim3(P::kThreads),  \
                       P::kLds, st,                                                            \
                       dz2, n, k, W2t, m, h1, x, F, part);                                     \
  } while (0)
  switch (nh) {
    case 1: MEPOL_L1B(1); break;
    case 2: MEPOL_L1B(2); break;
    case 3: MEPOL_L1B(3); break;
    default: MEPOL_L1B(4); break;
  }
#undef MEPOL_L1B
  MEPOL_CHECK_LAUNCH();
  const int64_t elems = (int64_t)m * (F + 1);
  double* grp = part + (size_t)nrb * elems;
  hipLaunchKernelGGL(mepol::gemm::layer1_reduce_kernel,
                     dim3((unsigned)((elems + 63) / 64), mepol::gemm::kGroups), dim3(256), 0, st,
                     part, nrb, m, F, grp);
  MEPOL_CHECK_LAUNCH();
  hipLaunchKernelGGL(mepol::gemm::layer1_reduce2_kernel, dim3((unsigned)((elems + 255) / 256)),
                     dim3(256), 0, st, grp, m, F, dW1, db1);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

extern "C" int mepol_dh1_layer1_backward(const double* dz2, int64_t n, int k, const double* W2t,
                                         int m, const double* h1, const double* x,
                                         int in_features, double* dW1, double* db1,
                                         void* workspace, size_t workspace_bytes, void* stream) {
  return dh1_layer1_backward<false>(dz2, n, k, W2t, m, h1, x, in_features, dW1, db1, workspace,
                                    workspace_bytes, stream);
}

extern "C" int mepol_dh1_layer1_backward_masked(const double* dz2, int64_t n, int k,
                                                const double* W2t, int m,
                                                const uint16_t* h1_mask, const double* x,
                                                int in_features, double* dW1, double* db1,
                                                void* workspace, size_t workspace_bytes,
                                                void* stream) {
  return dh1_layer1_backward<true>(dz2, n, k, W2t, m, h1_mask, x, in_features, dW1, db1,
                                   workspace, workspace_bytes, stream);
}

extern "C" int mepol_dh1_layer1_backward_w2(const double* dz2, int64_t n, int k, const double* W2,
                                            int m, const uint16_t* h1_mask, const double* x,
                                            int in_features, double* dW1, double* db1,
                                            void* workspace, size_t workspace_bytes,
                                            void* stream) {
  return dh1_layer1_backward<true, true>(dz2, n, k, W2, m, h1_mask, x, in_features, dW1, db1,
                                         workspace, workspace_bytes, stream);
}
