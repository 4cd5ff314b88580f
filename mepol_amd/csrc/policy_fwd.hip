// Fused forward of GaussianPolicy.get_log_p for the large-batch off-policy passes
// (src/policy.py:21-51: net = Linear(nf, h0) ReLU Linear(h0, h1) ReLU, mean = Linear(h1, a),
// logp = sum_a log N(act | mean, exp(log_std) + 1e-7)) as ONE kernel per 64-row block:
//
//   h1 = relu(x W1^T + b1)      f64 MFMA, K = nf (<= 64), a k-tile of h1 at a time, written to
//                               LDS as the next GEMM's A operand and to HBM (h1_out: the
//                               backward's dW2 operand and ReLU mask)
//   z2 = h1 W2^T                f64 MFMA (v_mfma_f64_16x16x4f64), 64 x 320 output tile per
//                               workgroup (8 waves, 32 x 80 each), K = h0 streamed in 16-tiles
//                               through double-buffered LDS; z2 (pre-bias) written to HBM for
//                               the head backward
//   mu = relu(z2 + b2) Wm^T + bm, logp   epilogue on the accumulators: per-lane partial mean
//                               over the lane's 5 columns, reduce-scatter over the 16 lanes of a
//                               row, fixed-order sum of the 4 column waves through LDS
//
// This replaces layer_forward + the z2 GEMM + head_forward (three passes over the N x h0 and
// N x h1 activations) with one: the layer-1 recompute costs ceil4(nf)/320 of the GEMM's MFMA
// work (10 % at nf = 29) and the head epilogue ~2 %.  Limits: nf <= 64, h1 (hidden[1]) <= 320.
//
// Round 5: with h0 even (every bench shape) the forward runs in a split form instead --
// layer1_kernel (h1 + its bit mask to HBM) then z2_head_kernel (the z2 GEMM with both operands
// read straight from L2 into the MFMA fragments: no LDS staging, no barrier in the K loop, and
// this kernel's head epilogue).  C3: 1.19 ms against 1.32 for the one-kernel form below, which
// stays for odd h0 (profiles/r5/f64/forward_split_ab.txt).
#include "common.hpp"

namespace mepol {
namespace pfwd {

constexpr int BM = 64, BN = 320;     // output tile (rows x h1 columns)
constexpr int WC = 4;                // column waves (80 columns each); 2 row waves (32 rows)
constexpr int FR = 2, FC = 5;        // 16x16 fragments per wave
constexpr int kThreads = 512;
constexpr int KT = 16, KP = 18;      // k-tile and padded LDS row (doubles)
constexpr int CB = BN * (KT / 2), PB = CB / kThreads;  // 16-B chunks of a W2 k-tile per thread
constexpr int kAChunk = 8;           // actions per epilogue pass
constexpr double kLog2Pi = 1.8378770664093453;
constexpr double kStdEps = 1e-7;
typedef double d4 __attribute__((ext_vector_type(4)));
static_assert(CB % kThreads == 0, "W2 k-tile chunks must divide the block");

template <int FP>
constexpr size_t lds_bytes() {
  return (2ull * BM * KP + 2ull * BN * KP + (size_t)(BM + 2 * KT) * (FP + 2)) * sizeof(double);
}

template <int FP, bool VEC>
__global__ __launch_bounds__(kThreads) void policy_fwd_kernel(
    const double* __restrict__ x, int64_t N, int F, const double* __restrict__ W1,
    const double* __restrict__ b1, int H1, const double* __restrict__ W2,
    const double* __restrict__ b2, int H2, const double* __restrict__ Wm,
    const double* __restrict__ bm, const double* __restrict__ log_std,
    const double* __restrict__ act, int A, double* __restrict__ h1_out,
    double* __restrict__ z2_out, double* __restrict__ mu_out, double* __restrict__ logp_out,
    uint16_t* __restrict__ mask_out) {
  constexpr int XP = FP + 2;  // padded x row: lanes of a fragment read hit distinct banks
  extern __shared__ double lds[];
  double* sA = lds;                    // [2][BM][KP]  h1 k-tile (A operand)
  double* sB = sA + 2 * BM * KP;       // [2][BN][KP]  W2 k-tile (B operand)
  double* sX = sB + 2 * BN * KP;       // [BM][XP]     x rows
  double* sW = sX + BM * XP;           // [2][KT][XP]  W1 rows of a k-tile (layer-1 B operand)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave / WC, wc = wave % WC;
  const int fr = lane & 15, g = lane >> 4;
  const int64_t row0 = (int64_t)blockIdx.x * BM;
  const int nkt = (H1 + KT - 1) / KT;

  // Operand loads below read a clamped (always valid) address and zero the value afterwards:
  // no branch around a load, so the compiler does not serialise them behind vmcnt waits.
  for (int e = tid; e < BM * FP; e += kThreads) {
    const int r = e / FP, f = e % FP;
    const int64_t rr = min<int64_t>(row0 + r, N - 1);
    const double v = x[rr * F + min(f, F - 1)];
    sX[r * XP + f] = (f < F && row0 + r < N) ? v : 0.0;
  }

  // ---- layer 1 on waves 0..3 (one per SIMD): rows 16 w .. 16 w + 15 of the block ----------
  // W1 rows of k-tile kt (16 x F): staged through LDS one tile ahead of the W2 tiles, so the
  // layer-1 waves issue no global loads of their own (a wait for one would also wait for the
  // h1 stores issued before it: vmcnt counts stores too)
  constexpr int PW = (KT * FP + kThreads - 1) / kThreads;
  double rw[PW];
  auto w1_load = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int e = tid + p * kThreads, r = e / FP, f = e % FP;
      rw[p] = W1[(int64_t)min(kt * KT + r, H1 - 1) * F + min(f, F - 1)];
    }
  };
  auto w1_store = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PW; ++p) {
      const int e = tid + p * kThreads, r = e / FP, f = e % FP;
      if (e < KT * FP) sW[((kt & 1) * KT + r) * XP + f] = (kt * KT + r < H1 && f < F) ? rw[p] : 0.0;
    }
  };
  auto h1_gen = [&](int kt, int buf) __attribute__((always_inline)) {
    // up to four independent MFMA chains (k-steps s mod 4) shorten the dependent latency.
    // (W1 rows >= H1 and columns >= F are zero in LDS)
    constexpr int NS = FP / 4, NCH = NS < 4 ? NS : 4;
    d4 hc[NCH];
#pragma unroll
    for (int u = 0; u < NCH; ++u) hc[u] = d4{0.0, 0.0, 0.0, 0.0};
    const double* xr = sX + (wave * 16 + fr) * XP + g;
    const double* wr1 = sW + ((kt & 1) * KT + fr) * XP + g;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      hc[s % NCH] = __builtin_amdgcn_mfma_f64_16x16x4f64(xr[4 * s], wr1[4 * s], hc[s % NCH], 0,
                                                         0, 0);
    d4 h = hc[0];
#pragma unroll
    for (int u = 1; u < NCH; ++u) h += hc[u];
    const int c = kt * KT + fr;
    const double bc = c < H1 ? b1[c] : 0.0;
    const int mw = (H1 + 15) / 16;  // mask row stride (16-bit words)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = wave * 16 + g + 4 * q;
      const double v = c < H1 ? fmax(h[q] + bc, 0.0) : 0.0;
      sA[(buf * BM + r) * KP + fr] = v;
      if (c < H1 && row0 + r < N) h1_out[(row0 + r) * H1 + c] = v;
      // relu'(h1) as bits for the backward (dh1's epilogue reads 2 B per 16 columns instead
      // of the 8-B h1 values): bit fr of word kt of row r = (h1[r][16 kt + fr] > 0)
      const uint64_t bits = __ballot(v > 0.0);
      if (mask_out && fr == 0 && row0 + r < N)
        mask_out[(row0 + r) * mw + kt] = (uint16_t)(bits >> (16 * g));
    }
  };

  // ---- W2 k-tiles: global -> registers -> LDS ---------------------------------------------
  double2 rb[PB];
  auto b_load = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int ch = tid + p * kThreads, r = ch >> 3, k = kt * KT + 2 * (ch & 7);
      const double* row = W2 + (int64_t)min(r, H2 - 1) * H1;
      double2 v;
      if constexpr (VEC)  // H1 even: k < H1 implies k + 1 < H1, 16-B aligned pair
        v = *reinterpret_cast<const double2*>(row + min(k, H1 - 2));
      else
        v = double2{row[min(k, H1 - 1)], row[min(k + 1, H1 - 1)]};
      rb[p] = v;  // masked in b_store: a select here would wait for the load at once
    }
  };
  auto b_store = [&](int kt, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int p = 0; p < PB; ++p) {
      const int ch = tid + p * kThreads, r = ch >> 3, k = kt * KT + 2 * (ch & 7);
      double2 v = rb[p];
      if (r >= H2 || k >= H1) v = double2{0.0, 0.0};
      if (k + 1 >= H1) v.y = 0.0;
      *reinterpret_cast<double2*>(sB + (buf * BN + r) * KP + 2 * (ch & 7)) = v;
    }
  };

  d4 acc[FR][FC];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < FC; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};

  b_load(0);
  w1_load(0);
  w1_store(0);
  if (nkt > 1) {
    w1_load(1);
    w1_store(1);
  }
  __syncthreads();  // sX, sW
  if (wave < 4) h1_gen(0, 0);
  b_store(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nkt) {
      b_load(kt + 1);
      if (kt + 2 < nkt) w1_load(kt + 2);
      // layer 1 of the NEXT k-tile ahead of this tile's GEMM, so its short dependent MFMA
      // chains, bias/ReLU and HBM stores overlap the GEMM instead of stalling the barrier.
      // sA[buf ^ 1] was last read in iteration kt - 1, behind that iteration's barrier.
      if (wave < 4) h1_gen(kt + 1, buf ^ 1);
    }
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
    if (kt + 1 < nkt) {
      b_store(kt + 1, buf ^ 1);
      if (kt + 2 < nkt) w1_store(kt + 2);  // sW[kt & 1]: last read by h1_gen(kt), a barrier ago
    }
    __syncthreads();
  }

  // ---- epilogue: z2 out, then the head on relu(z2 + b2) -----------------------------------
  // C/D map of the f64 16x16x4 MFMA: col = lane & 15, row = (lane >> 4) + 4 q.
  double b2v[FC];
#pragma unroll
  for (int j = 0; j < FC; ++j) {
    const int c = wc * FC * 16 + j * 16 + fr;
    b2v[j] = c < H2 ? b2[c] : 0.0;
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + wr * FR * 16 + i * 16 + g + 4 * q;
        if (c < H2 && r < N) z2_out[r * H2 + c] = acc[i][j][q];
      }
  }
  double* sMu = sB;  // [WC][BM][kAChunk]; the loop's last barrier retired every sB read
  const int er = tid >> 3, ea = tid & 7;  // combine step: row er of the block, action slot ea
  double lp = 0.0;
  for (int a0 = 0; a0 < A; a0 += kAChunk) {
    double wmv[FC][kAChunk];
#pragma unroll
    for (int j = 0; j < FC; ++j) {
      const int c = wc * FC * 16 + j * 16 + fr;
#pragma unroll
      for (int a = 0; a < kAChunk; ++a)
        wmv[j][a] = (c < H2 && a0 + a < A) ? Wm[(int64_t)(a0 + a) * H2 + c] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double p[kAChunk];
#pragma unroll
        for (int a = 0; a < kAChunk; ++a) p[a] = 0.0;
#pragma unroll
        for (int j = 0; j < FC; ++j) {
          const double rv = fmax(acc[i][j][q] + b2v[j], 0.0);
#pragma unroll
          for (int a = 0; a < kAChunk; ++a) p[a] = fma(rv, wmv[j][a], p[a]);
        }
        // reduce-scatter over the 16 lanes of the row: halving exchanges on lane bits 8, 4, 2
        // leave lane l with component ((l>>3)&1)*4 + ((l>>2)&1)*2 + ((l>>1)&1), then bit 1
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const bool up = (fr & 8) != 0;
          const double send = up ? p[a] : p[a + 4];
          p[a] = (up ? p[a + 4] : p[a]) + __shfl_xor(send, 8, kWave);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const bool up = (fr & 4) != 0;
          const double send = up ? p[a] : p[a + 2];
          p[a] = (up ? p[a + 2] : p[a]) + __shfl_xor(send, 4, kWave);
        }
        {
          const bool up = (fr & 2) != 0;
          const double send = up ? p[0] : p[1];
          p[0] = (up ? p[1] : p[0]) + __shfl_xor(send, 2, kWave);
        }
        p[0] += __shfl_xor(p[0], 1, kWave);
        const int comp = ((fr >> 3) & 1) * 4 + ((fr >> 2) & 1) * 2 + ((fr >> 1) & 1);
        if ((fr & 1) == 0) {
          const int rl = wr * FR * 16 + i * 16 + g + 4 * q;
          sMu[(wc * BM + rl) * kAChunk + comp] = p[0];
        }
      }
    __syncthreads();
    {
      const int a = a0 + ea;
      const int64_t r = row0 + er;
      double term = 0.0;
      if (a < A && r < N) {
        double m = sMu[(0 * BM + er) * kAChunk + ea];
#pragma unroll
        for (int w = 1; w < WC; ++w) m += sMu[(w * BM + er) * kAChunk + ea];
        m += bm[a];
        const double lsa = log_std[a];
        const double sd = exp(lsa) + kStdEps;
        const double d = act[r * A + a] - m;
        mu_out[r * A + a] = m;
        term = -0.5 * (kLog2Pi + 2.0 * lsa + d * d / (sd * sd));
      }
      term += __shfl_xor(term, 4, kWave);
      term += __shfl_xor(term, 2, kWave);
      term += __shfl_xor(term, 1, kWave);
      lp += term;
    }
    __syncthreads();
  }
  if (ea == 0 && row0 + er < N) logp_out[row0 + er] = lp;
}

// ---------------------------------------------------------------------------------------
// Split form (hidden0 even): layer 1 alone, then z2 + head with no LDS operand staging.
// ---------------------------------------------------------------------------------------
// h1 = relu(x W1^T + b1) and its bit mask, one wave per RG groups of 16 rows: the rows' x
// fragments stay in registers (k = 4 s + g), the 16-column tiles of W1 stream from L2 with the
// next tile's fragment loaded under the current tile's MFMAs (RG independent accumulation chains
// of NS steps), stores are whole 128-B row segments.  HBM-write bound (h1 is N x h0 f64).
// Round 6: RG = 2 (was one row group per wave and no prefetch: every wave re-read all of W1
// through L1 per 16 rows, 1.3 GB per call at C3, and waited for each tile).
template <int FP, int RG>
__global__ __launch_bounds__(256) void layer1_kernel(const double* __restrict__ x, int64_t N,
                                                     int F, const double* __restrict__ W1,
                                                     const double* __restrict__ b1, int H1,
                                                     double* __restrict__ h1_out,
                                                     uint16_t* __restrict__ mask_out) {
  constexpr int NS = FP / 4;
  const int l = threadIdx.x & 63, fr = l & 15, g = l >> 4;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 * RG;
  if (r0 >= N) return;  // wave-uniform
  double xv[RG][NS];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    const int64_t xr = min<int64_t>(r0 + 16 * rg + fr, N - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int f = 4 * s + g;
      const double v = x[xr * F + min(f, F - 1)];
      xv[rg][s] = f < F ? v : 0.0;
    }
  }
  const int nkt = (H1 + 15) / 16, mw = nkt;
  double wv[2][NS], bc[2];
  auto loadw = [&](int b, int kt) __attribute__((always_inline)) {
    const int c = min(kt * 16 + fr, H1 - 1);
    const double* wr = W1 + (int64_t)c * F;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int f = 4 * s + g;
      const double v = wr[min(f, F - 1)];
      wv[b][s] = f < F ? v : 0.0;
    }
    bc[b] = b1[c];
  };
  auto tile = [&](int b, int kt) __attribute__((always_inline)) {
    if (kt + 1 < nkt) loadw(b ^ 1, kt + 1);  // uniform
    d4 h[RG];
#pragma unroll
    for (int rg = 0; rg < RG; ++rg) h[rg] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int rg = 0; rg < RG; ++rg)
        h[rg] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[rg][s], wv[b][s], h[rg], 0, 0, 0);
    const int c = kt * 16 + fr;
#pragma unroll
    for (int rg = 0; rg < RG; ++rg)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = r0 + 16 * rg + g + 4 * q;
        const double v = c < H1 ? fmax(h[rg][q] + bc[b], 0.0) : 0.0;
        // streaming (nontemporal) store: h1 (640 MB at C3) is far past L2 / MALL; 209 -> 204 us
        if (c < H1 && r < N) __builtin_nontemporal_store(v, h1_out + r * H1 + c);
        const uint64_t bits = __ballot(v > 0.0);
        if (mask_out && fr == 0 && r < N) mask_out[r * mw + kt] = (uint16_t)(bits >> (16 * g));
      }
  };
  loadw(0, 0);
  int kt = 0;
#pragma nounroll
  for (; kt + 1 < nkt; kt += 2) {
    tile(0, kt);
    tile(1, kt + 1);
  }
  if (kt < nkt) tile(0, kt);
}

// z2 = h1 W2^T and the head, one workgroup per 64-row block: wave w owns columns
// [80 w, 80 w + 80) (4 x 5 fragments) and reads both operands straight from L2 into the MFMA
// fragments -- a lane takes 16 B of its row per fragment, k = 8 st + 2 g + {0, 1}, and the
// stage's two k-steps use the two halves (h1 and W2 in the same k order).  No LDS staging and
// no barrier in the K loop; the head epilogue is the fused kernel's (LDS only for the sum of
// the 4 column waves).  tools/z2_probe.py: the bare GEMM at 50.7 TF/s (C3) against 45 in the
// fused kernel's k-tile loop.
namespace zh {
constexpr int FO = 4, FI = 5, NW = 4, NS = 2, NL = FO + FI;
constexpr int BM = 16 * FO;  // rows per workgroup (x 320 columns)
}  // namespace zh

__global__ __launch_bounds__(64 * zh::NW) __attribute__((amdgpu_waves_per_eu(2))) void z2_head_kernel(
    const double* __restrict__ h1, int64_t N, int H1, const double* __restrict__ W2,
    const double* __restrict__ b2, int H2, const double* __restrict__ Wm,
    const double* __restrict__ bm, const double* __restrict__ log_std,
    const double* __restrict__ act, int A, double* __restrict__ z2_out,
    double* __restrict__ mu_out, double* __restrict__ logp_out) {
  constexpr int FO = zh::FO, FI = zh::FI, NW = zh::NW, NS = zh::NS, NL = zh::NL, ZM = zh::BM;
  __shared__ double sMu[NW * ZM * 4];
  const int tid = threadIdx.x, l = tid & 63, fr = l & 15, g = l >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t row0 = (int64_t)blockIdx.x * ZM;
  const int col0 = 16 * FI * w;
  const double* ap[FO];
  const double* bp[FI];
#pragma unroll
  for (int t = 0; t < FO; ++t) ap[t] = h1 + min<int64_t>(row0 + 16 * t + fr, N - 1) * H1 + 2 * g;
#pragma unroll
  for (int u = 0; u < FI; ++u) bp[u] = W2 + (int64_t)min(col0 + 16 * u + fr, H2 - 1) * H1 + 2 * g;
  d4 acc[FO][FI];
#pragma unroll
  for (int t = 0; t < FO; ++t)
#pragma unroll
    for (int u = 0; u < FI; ++u) acc[t][u] = d4{0.0, 0.0, 0.0, 0.0};
  // stage st reads k = 8 st + 2 g (+1); H1 is even, so a pair is whole or past the end.  The
  // address is clamped to the last pair and the tail stage's pairs past H1 are zeroed at use.
  const int nst = (H1 + 7) / 8, nfull = H1 / 8;
  double2 R[NS][NL];
  auto load = [&](double2 (&D)[NL], int st) __attribute__((always_inline)) {
    const int k = min(8 * st, H1 - 2 - 2 * g);  // k + 2 g <= H1 - 2
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
      if (st + p >= nfull && 8 * (st + p) + 2 * g >= H1) {  // the tail stage's missing pairs
#pragma unroll
        for (int v = 0; v < NL; ++v) R[p][v] = double2{0.0, 0.0};
      }
      mma(R[p]);
    }
  }

  // ---- epilogue: z2 out, then the head on relu(z2 + b2) (as policy_fwd_kernel's) ----------
  double b2v[FI];
#pragma unroll
  for (int u = 0; u < FI; ++u) {
    const int c = col0 + 16 * u + fr;
    b2v[u] = c < H2 ? b2[c] : 0.0;
#pragma unroll
    for (int t = 0; t < FO; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = row0 + 16 * t + g + 4 * q;
        if (c < H2 && r < N) z2_out[r * H2 + c] = acc[t][u][q];
      }
  }
  // 4 actions per pass (the fused kernel's 8 would hold 40 more registers next to the 160 of
  // the accumulators): reduce-scatter over lane bits 8 and 4, sum over bits 2 and 1
  constexpr int AC = 4;
  const int er = tid >> 2, ea = tid & 3;  // combine step: row er of the block, action slot ea
  double lp = 0.0;
  for (int a0 = 0; a0 < A; a0 += AC) {
    double wmv[FI][AC];
#pragma unroll
    for (int u = 0; u < FI; ++u) {
      const int c = col0 + 16 * u + fr;
#pragma unroll
      for (int a = 0; a < AC; ++a)
        wmv[u][a] = (c < H2 && a0 + a < A) ? Wm[(int64_t)(a0 + a) * H2 + c] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < FO; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double p[AC];
#pragma unroll
        for (int a = 0; a < AC; ++a) p[a] = 0.0;
#pragma unroll
        for (int u = 0; u < FI; ++u) {
          const double rv = fmax(acc[t][u][q] + b2v[u], 0.0);
#pragma unroll
          for (int a = 0; a < AC; ++a) p[a] = fma(rv, wmv[u][a], p[a]);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const bool up = (fr & 8) != 0;
          const double send = up ? p[a] : p[a + 2];
          p[a] = (up ? p[a + 2] : p[a]) + __shfl_xor(send, 8, kWave);
        }
        {
          const bool up = (fr & 4) != 0;
          const double send = up ? p[0] : p[1];
          p[0] = (up ? p[1] : p[0]) + __shfl_xor(send, 4, kWave);
        }
        p[0] += __shfl_xor(p[0], 2, kWave);
        p[0] += __shfl_xor(p[0], 1, kWave);
        const int comp = ((fr >> 3) & 1) * 2 + ((fr >> 2) & 1);
        if ((fr & 3) == 0) sMu[(w * ZM + 16 * t + g + 4 * q) * AC + comp] = p[0];
      }
    __syncthreads();
    {
      const int a = a0 + ea;
      const int64_t r = row0 + er;
      double term = 0.0;
      if (a < A && r < N) {
        double m = sMu[(0 * ZM + er) * AC + ea];
#pragma unroll
        for (int v = 1; v < NW; ++v) m += sMu[(v * ZM + er) * AC + ea];
        m += bm[a];
        const double lsa = log_std[a];
        const double sd = exp(lsa) + kStdEps;
        const double d = act[r * A + a] - m;
        mu_out[r * A + a] = m;
        term = -0.5 * (kLog2Pi + 2.0 * lsa + d * d / (sd * sd));
      }
      term += __shfl_xor(term, 2, kWave);
      term += __shfl_xor(term, 1, kWave);
      lp += term;
    }
    __syncthreads();
  }
  if (ea == 0 && row0 + er < N) logp_out[row0 + er] = lp;
}

#ifndef MEPOL_L1_RG
#define MEPOL_L1_RG 2
#endif
constexpr int kLayer1RowGroups = MEPOL_L1_RG;  // row groups of 16 per wave (layer1_kernel)

template <int FP>
int launch_split(const double* x, int64_t n, int F, const double* W1, const double* b1, int H1,
                 const double* W2, const double* b2, int H2, const double* Wm, const double* bm,
                 const double* log_std, const double* act, int A, double* h1, double* z2,
                 double* mu, double* logp, uint16_t* mask, hipStream_t st) {
  const unsigned blocks = (unsigned)((n + 63) / 64);
  constexpr int RG = kLayer1RowGroups;
  hipLaunchKernelGGL((layer1_kernel<FP, RG>), dim3((unsigned)((n + 64 * RG - 1) / (64 * RG))),
                     dim3(256), 0, st, x, n, F, W1, b1, H1, h1, mask);
  MEPOL_CHECK_LAUNCH();
  hipLaunchKernelGGL(z2_head_kernel, dim3(blocks), dim3(64 * zh::NW), 0, st, h1, n, H1, W2, b2,
                     H2, Wm, bm, log_std, act, A, z2, mu, logp);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

template <int FP, bool VEC>
int launch(const double* x, int64_t n, int F, const double* W1, const double* b1, int H1,
           const double* W2, const double* b2, int H2, const double* Wm, const double* bm,
           const double* log_std, const double* act, int A, double* h1, double* z2, double* mu,
           double* logp, uint16_t* mask, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    MEPOL_HIP(hipFuncSetAttribute((const void*)policy_fwd_kernel<FP, VEC>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds_bytes<FP>()));
    attr = true;
  }
  const unsigned blocks = (unsigned)((n + BM - 1) / BM);
  hipLaunchKernelGGL((policy_fwd_kernel<FP, VEC>), dim3(blocks), dim3(kThreads), lds_bytes<FP>(), st,
                     x, n, F, W1, b1, H1, W2, b2, H2, Wm, bm, log_std, act, A, h1, z2, mu, logp,
                     mask);
  MEPOL_CHECK_LAUNCH();
  return 0;
}

}  // namespace pfwd
}  // namespace mepol

static int policy_forward(const double* x, int64_t n, int in_features, const double* W1,
                          const double* b1, int hidden0, const double* W2, const double* b2,
                          int hidden1, const double* Wm, const double* bm,
                          const double* log_std, const double* actions, int action_dim,
                          double* h1_out, double* z2_out, double* mu_out, double* logp_out,
                          uint16_t* h1_mask_out, void* stream) {
  using namespace mepol::pfwd;
  if (n < 0 || in_features <= 0 || in_features > 64 || hidden0 <= 0 || hidden1 <= 0 ||
      hidden1 > BN || action_dim <= 0 || !x || !W1 || !b1 || !W2 || !b2 || !Wm || !bm ||
      !log_std || !actions || !h1_out || !z2_out || !mu_out || !logp_out ||
      ((uintptr_t)W2 & 15)) {
    mepol::set_error("mepol_policy_forward: bad arguments (in_features <= 64, hidden1 <= %d)",
                     BN);
    return mepol::kErrBadArg;
  }
  if (n == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  // the split form (layer1_kernel + z2_head_kernel) needs 16-B aligned h1 rows; C3 forward
  // 1.19 ms against the one-kernel form's 1.32 (profiles/r5/f64/forward_split_ab.txt)
  const bool split = hidden0 % 2 == 0 && ((uintptr_t)h1_out & 15) == 0;
#define MEPOL_PF(FPV)                                                                        \
  {                                                                                          \
  if (split)                                                                                 \
    return launch_split<FPV>(x, n, in_features, W1, b1, hidden0, W2, b2, hidden1, Wm, bm,     \
                             log_std, actions, action_dim, h1_out, z2_out, mu_out, logp_out, \
                             h1_mask_out, st);                                               \
  return (hidden0 % 2 == 0 && hidden0 >= 2)                                                  \
             ? launch<FPV, true>(x, n, in_features, W1, b1, hidden0, W2, b2, hidden1, Wm, bm, \
                                 log_std, actions, action_dim, h1_out, z2_out, mu_out,        \
                                 logp_out, h1_mask_out, st)                                   \
             : launch<FPV, false>(x, n, in_features, W1, b1, hidden0, W2, b2, hidden1, Wm,    \
                                  bm, log_std, actions, action_dim, h1_out, z2_out, mu_out,   \
                                  logp_out, h1_mask_out, st);                                  \
  }
  if (in_features <= 4) MEPOL_PF(4);
  if (in_features <= 8) MEPOL_PF(8);
  if (in_features <= 16) MEPOL_PF(16);
  if (in_features <= 32) MEPOL_PF(32);
  if (in_features <= 48) MEPOL_PF(48);
  MEPOL_PF(64);
#undef MEPOL_PF
}

extern "C" int mepol_policy_forward(const double* x, int64_t n, int in_features,
                                    const double* W1, const double* b1, int hidden0,
                                    const double* W2, const double* b2, int hidden1,
                                    const double* Wm, const double* bm, const double* log_std,
                                    const double* actions, int action_dim, double* h1_out,
                                    double* z2_out, double* mu_out, double* logp_out,
                                    void* stream) {
  return policy_forward(x, n, in_features, W1, b1, hidden0, W2, b2, hidden1, Wm, bm, log_std,
                        actions, action_dim, h1_out, z2_out, mu_out, logp_out, nullptr, stream);
}

extern "C" int mepol_policy_forward_masked(const double* x, int64_t n, int in_features,
                                           const double* W1, const double* b1, int hidden0,
                                           const double* W2, const double* b2, int hidden1,
                                           const double* Wm, const double* bm,
                                           const double* log_std, const double* actions,
                                           int action_dim, double* h1_out, double* z2_out,
                                           double* mu_out, double* logp_out,
                                           uint16_t* h1_mask_out, void* stream) {
  if (!h1_mask_out) {
    mepol::set_error("mepol_policy_forward_masked: h1_mask_out is null");
    return mepol::kErrBadArg;
  }
  return policy_forward(x, n, in_features, W1, b1, hidden0, W2, b2, hidden1, Wm, bm, log_std,
                        actions, action_dim, h1_out, z2_out, mu_out, logp_out, h1_mask_out,
                        stream);
}
