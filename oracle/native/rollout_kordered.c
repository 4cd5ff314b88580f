/* CPU restatement of collect_particles (src/algorithms/mepol.py:76-109) for the reference's
 * 2 -> [h0, h1] -> a ReLU GaussianPolicy (src/policy.py:21-28, 53-61) on MountainCar
 * (src/envs/mountain_car_wall.py:13-45) / GridWorld (src/envs/gridworld_continuous.py:128-154),
 * with the policy MLP summed in ONE documented order -- TEST INFRASTRUCTURE ONLY (the parity
 * oracle; tests/ load it through oracle/mepol_oracle.py, the product never does).
 *
 * The reference's matmul order is MKL's and cannot be matched; this order is the one the HIP
 * rollout kernels (mepol_amd/csrc/envs.hip) commit to, so their actions can be compared bit for
 * bit instead of to ~1e-15:
 *   h1_c  = max((x0 * W1[c][0] + x1 * W1[c][1]) + b1[c], 0)         each op rounded
 *   h2_j  = max(((c_0 + c_1) + ...) + b2[j], 0),  c_r = fma-chain_k(W2[j][k] * h1_k) over
 *           k in [r L, min(r L + L, h0)), L = ceil(h0 / k_chunks), r = 0 .. k_chunks - 1
 *           (k_chunks = 1: one chain over all rows; the multi-workgroup kernel uses 4)
 *   part_w[a] = xor-butterfly sum (strides 32, 16, .., 1; lane 0's value) of Wm[a][j] * h2_j over
 *               the 64 columns j of wave w (zero past h1), w = 0 .. ceil(max(h0,h1)/64) - 1
 *   mu[a] = ((part_0 + part_1) + ...) + bm[a];  a = mu + noise * sd   (policy.py:59)
 * Built with -ffp-contract=off; fma() is glibc's correctly rounded fma. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void mc_step(double* p, double* v, double a0) {
  const double force = fmin(fmax(a0, -1.0), 1.0);
  *v = *v + (force * 0.0015 - 0.0025 * cos(3.0 * *p));
  if (*v > 0.07) *v = 0.07;
  if (*v < -0.07) *v = -0.07;
  *p = *p + *v;
  if (*p > 0.6) *p = 0.6;
  if (*p < -1.2) *p = -1.2;
  if (*p == -1.2 && *v < 0) *v = 0.0;
  if (*p > 0.45) {
    *p = 0.45;
    *v = 0.0;
  }
}

static int inside(double x, double y, double x0, double x1, double y0, double y1) {
  return x0 <= x && x <= x1 && y0 <= y && y <= y1;
}

static void gw_step(float* sx, float* sy, double ax, double ay) {
  const double dx = fmin(fmax(ax, -0.2), 0.2), dy = fmin(fmax(ay, -0.2), 0.2);
  const double x = (double)*sx, y = (double)*sy;
  double nx = x + dx, ny = y + dy;
  const double h = 1.25, w = 2.5, D = 6.0;
  int hit = inside(nx, ny, -h, h, -w, w) || inside(nx, ny, -w, -h, -h, h) ||
            inside(nx, ny, h, w, -h, h) || inside(nx, ny, -D, -(D - w), -h, h) ||
            inside(nx, ny, -h, h, -D, -(D - w)) || inside(nx, ny, D - w, D, -h, h) ||
            inside(nx, ny, -h, h, D - w, D);
  if (hit || fabs(nx) >= D || fabs(ny) >= D) {
    nx = x;
    ny = y;
  }
  *sx = (float)nx;
  *sy = (float)ny;
}

/* mean [a_dim] of one state in the order above */
static void mlp_mean(double x0, double x1, int h0, int h1, int a_dim, int k_chunks,
                     const double* W1,
                     const double* b1, const double* W2, const double* b2, const double* Wm,
                     const double* bm, double* hid1, double* hid2, double* mu) {
  for (int c = 0; c < h0; ++c) hid1[c] = fmax((x0 * W1[2 * c] + x1 * W1[2 * c + 1]) + b1[c], 0.0);
  for (int j = 0; j < h1; ++j) {
    const int L = (h0 + k_chunks - 1) / k_chunks;
    double acc = 0.0;
    for (int r = 0; r < k_chunks; ++r) {
      const int kb = r * L < h0 ? r * L : h0, ke = kb + L < h0 ? kb + L : h0;
      double c = 0.0;
      for (int k = kb; k < ke; ++k) c = fma(W2[(int64_t)j * h0 + k], hid1[k], c);
      acc = (r == 0) ? c : acc + c;
    }
    hid2[j] = fmax(acc + b2[j], 0.0);
  }
  const int hmax = h0 > h1 ? h0 : h1;
  const int nw = (hmax + 63) / 64;
  for (int a = 0; a < a_dim; ++a) {
    double m = 0.0;
    for (int w = 0; w < nw; ++w) {
      double v[64];
      for (int l = 0; l < 64; ++l) {
        const int j = 64 * w + l;
        v[l] = (j < h1) ? Wm[(int64_t)a * h1 + j] * hid2[j] : 0.0 * 0.0;
      }
      for (int s = 32; s >= 1; s >>= 1) {
        double nv[64];
        for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ s];
        memcpy(v, nv, sizeof(v));
      }
      m = (w == 0) ? v[0] : m + v[0];
    }
    mu[a] = m + bm[a];
  }
}

/* env 0 = MountainCar (init64 [n][2]), 1 = GridWorld (init32 [n][2]); noise [T][n][a_dim];
 * W2 [h1][h0] (nn.Linear layout); states [n][T+1][2] f32, actions [n][T][a_dim] f32. */
int rollout_kordered(int env, int64_t n, int64_t T, int h0, int h1, int a_dim, int k_chunks,
                     const double* W1,
                     const double* b1, const double* W2, const double* b2, const double* Wm,
                     const double* bm, const double* sd, const double* init64,
                     const float* init32, const double* noise, float* states, float* actions) {
  if (a_dim > 8 || h0 <= 0 || h1 <= 0 || k_chunks <= 0) return 1;
  double* hid1 = (double*)malloc(sizeof(double) * h0);
  double* hid2 = (double*)malloc(sizeof(double) * h1);
  for (int64_t i = 0; i < n; ++i) {
    double p = 0, v = 0, x0, x1;
    float gx = 0, gy = 0;
    if (env == 0) {
      p = init64[2 * i];
      v = init64[2 * i + 1];
      x0 = p;
      x1 = v;
    } else {
      gx = init32[2 * i];
      gy = init32[2 * i + 1];
      x0 = gx;
      x1 = gy;
    }
    states[(i * (T + 1)) * 2] = (float)x0;
    states[(i * (T + 1)) * 2 + 1] = (float)x1;
    for (int64_t t = 0; t < T; ++t) {
      double mu[8], act[8];
      mlp_mean(x0, x1, h0, h1, a_dim, k_chunks, W1, b1, W2, b2, Wm, bm, hid1, hid2, mu);
      for (int a = 0; a < a_dim; ++a) {
        act[a] = mu[a] + noise[(t * n + i) * a_dim + a] * sd[a];
        actions[(i * T + t) * a_dim + a] = (float)act[a];
      }
      if (env == 0) {
        mc_step(&p, &v, act[0]);
        x0 = p;
        x1 = v;
      } else {
        gw_step(&gx, &gy, act[0], act[1]);
        x0 = gx;
        x1 = gy;
      }
      states[(i * (T + 1) + t + 1) * 2] = (float)x0;
      states[(i * (T + 1) + t + 1) * 2 + 1] = (float)x1;
    }
  }
  free(hid1);
  free(hid2);
  return 0;
}
