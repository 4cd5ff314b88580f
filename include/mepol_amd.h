/* mepol_amd.h -- C ABI of the MI355X (gfx950) MEPOL hot path.
 *
 * The reference (RiccZamboni/mepol) is pure Python and has no FFI; these entry points are what
 * its hot path (src/algorithms/mepol.py) binds to when it is switched to this library.  Each
 * function names the reference interface it replaces.  The Python drop-in module
 * (mepol_amd/algorithms/mepol.py) calls them through ctypes (mepol_amd/_lib.py); the binding a
 * maintainer would add to the reference is shown in INTEGRATION.md.
 *
 * Conventions
 *  - All array arguments are DEVICE pointers owned by the caller (e.g. torch tensors via
 *    data_ptr()); nothing is allocated inside a call.  Scratch comes from a caller-owned
 *    workspace whose size the *_workspace_size query returns.
 *  - `stream` is a hipStream_t; every call only enqueues work on it (no host sync), so calls
 *    can be captured into a hipGraph -- with ONE exception: mepol_knn synchronises `stream`
 *    once per call to validate its input before the scan (sklearn raises on NaN / inf);
 *    mepol_knn_deferred is the same call with the validation result left on the device, and
 *    never blocks.  The per-iteration entry points (entropy, IW, head, GEMMs, optimizer)
 *    never synchronise.
 *  - Return value: 0 on success, a hipError_t value or one of the MEPOL_ERR_* codes otherwise;
 *    mepol_last_error_string() describes the last failure of the calling thread.
 *  - Stateless and re-entrant; ordering comes from the stream.
 *  - Particle indices are int32 on device (N < 2^31); the Python boundary widens them to the
 *    reference's int64 where it returns them.
 */
#ifndef MEPOL_AMD_H
#define MEPOL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped on every incompatible change of the signatures below (2: mepol_rollout_mlp takes a
 * workspace; mepol_gemm_dpp removed; 3: mepol_iw_normalize_gathered takes the per-rank
 * trajectory sums).  mepol_abi_version() returns the library's value. */
#define MEPOL_ABI_VERSION 4

#define MEPOL_ERR_BAD_ARG 1001
#define MEPOL_ERR_WORKSPACE 1002
#define MEPOL_ERR_UNSUPPORTED 1003

const char* mepol_last_error_string(void);
int mepol_abi_version(void);
/* Stream-ordered copy (device <-> pinned host / device); captured as a graph memcpy node. */
int mepol_memcpy_async(void* dst, const void* src, size_t bytes, void* stream);


/* ---- k-NN ---------------------------------------------------------------------------------
 * Replaces src/algorithms/mepol.py:190-192
 *     NearestNeighbors(n_neighbors=k+1, metric='euclidean', algorithm='auto', n_jobs=W)
 *         .fit(next_states).kneighbors(next_states)
 * cand [n_cand, d] f32 row-major, query [n_query, d] f32 (a shard of cand or cand itself).
 * Outputs: dist_out [n_query, kp1] f64 = sqrt(sum_f (q_f - c_f)^2) in f64 (sklearn kd_tree's
 * arithmetic), rows ascending, ties by smaller index; idx_out [n_query, kp1] int64 (nullable);
 * idx32_out [kp1, n_query] int32 TRANSPOSED (nullable; the layout the entropy kernels read).
 * n_fallback_out (nullable, device int32): number of queries answered by the exhaustive path.
 * split_hint: 0 = automatic candidate split.  Any d >= 1 and any 1 <= kp1 <= n_cand (sklearn
 * raises for kp1 > n_samples; so does this, MEPOL_ERR_BAD_ARG); n_cand < 2^31 - 64.  Plans:
 * d <= 63 and kp1 <= 60 run the f16 MFMA screen + certified f64 re-rank (queries it cannot
 * certify take the exhaustive scan); every other shape, and any input with a row whose f32
 * squared norm overflows (the screen cannot scale it), is answered by the exhaustive f64 scan
 * for every query (mepol_knn_plan_info reports *ks = 0 for such a plan).
 * Input validation (sklearn's check_array in fit/kneighbors): a NaN / inf coordinate in cand or
 * query returns MEPOL_ERR_BAD_ARG ("Input contains NaN or infinity").  The check synchronises
 * `stream` once per call (before the scan is launched), as the reference's kneighbors call
 * blocks. */
int mepol_knn_workspace_size(int64_t n_cand, int64_t n_query, int d, int kp1, int split_hint,
                             size_t* bytes);
/* Plan of a call: *ks = 10 * (k-steps of 16) + candidate halves (1: f16 hi only, 2: hi + lo),
 * *list = per-half selection list length, *split = candidate ranges; an exhaustive plan
 * reports *ks = 0, *split = 0 and *list = its block-select capacity. */
int mepol_knn_plan_info(int64_t n_cand, int64_t n_query, int d, int kp1, int split_hint, int* ks,
                        int* list, int* split);
int mepol_knn(const float* cand, int64_t n_cand, const float* query, int64_t n_query, int d,
              int kp1, int split_hint, double* dist_out, int64_t* idx_out, int32_t* idx32_out,
              int32_t* n_fallback_out, void* workspace, size_t workspace_bytes, void* stream);
/* mepol_knn without the host synchronisation: invalid_out (device int32 [2], required) receives
 * [rows with a NaN / inf coordinate, rows whose squared norm overflows f32] in stream order.
 * When the first is nonzero every later kernel of the call returns at once (the outputs are
 * then undefined); the caller reads invalid_out at its next synchronisation point and raises
 * as mepol_knn would (the epoch path does so once the CSR build is queued behind the k-NN).
 * The second is informational: such a call is answered by the exhaustive scan. */
int mepol_knn_deferred(const float* cand, int64_t n_cand, const float* query, int64_t n_query,
                       int d, int kp1, int split_hint, double* dist_out, int64_t* idx_out,
                       int32_t* idx32_out, int32_t* n_fallback_out, int32_t* invalid_out,
                       void* workspace, size_t workspace_bytes, void* stream);
/* Exhaustive f64 scan for every query, no validation, no workspace (an independent check of
 * mepol_knn); kp1 <= 3072 (beyond: MEPOL_ERR_UNSUPPORTED, mepol_knn takes any kp1);
 * scratch_idx is unused (nullable). */
int mepol_knn_exact(const float* cand, int64_t n_cand, const float* query, int64_t n_query, int d,
                    int kp1, double* dist_out, int64_t* idx_out, int32_t* idx32_out,
                    int32_t* scratch_idx, void* stream);

/* ---- importance weights -------------------------------------------------------------------
 * Replaces compute_importance_weights, src/algorithms/mepol.py:114-139:
 *   u[off[n]+t] = exp(cumsum_{s<=t}(logp_t - logp_b)[n, s]);  w = u / sum(u).
 * logp_t/logp_b: [num_traj, T_stride] f64 (log-probs of target / behavioral policy);
 * traj_offsets: [num_traj+1] int64 particle offsets (real trajectory lengths, mepol.py:122).
 * traj_sum_out [num_traj]; w_out/U_out nullable (skip normalisation, e.g. multi-rank). */
int mepol_iw_forward(const double* logp_t, const double* logp_b, int64_t num_traj,
                     int64_t T_stride, const int64_t* traj_offsets, int64_t n_particles,
                     double* u_out, double* traj_sum_out, double* w_out, double* U_out,
                     void* stream);
/* w = u / *U with a device scalar U (multi-rank: U all-reduced). */
int mepol_iw_normalize(const double* u, const double* U, int64_t n, double* w, void* stream);

/* ---- entropy / KL -------------------------------------------------------------------------
 * Replaces compute_entropy (mepol.py:142-154) and compute_kl (mepol.py:157-174), fused:
 *   W_i = sum_{c<k} w[I[i,c]];  V_i = D[i,k]^ns pi^(ns/2)/G;
 *   out4[0] = H  = -sum_i (W_i/k) log(W_i/(V_i+eps)+eps) + B
 *   out4[1] = KL = (1/n_w) sum_i log(k/(n_w W_i) + eps)     (before the max(0, .) clamp)
 *   out4[2], out4[3] = the two raw sums (for cross-rank reduction).
 * w [n_w] (global), idxT [kp1, n] int32, D [n, kp1] f64; W_out, g_out [n] (g = dH/dW);
 * partials: [2 * mepol_entropy_partials_size(n)] f64 scratch. */
int mepol_entropy_partials_size(int64_t n_particles);
int mepol_entropy_forward(const double* w, const int32_t* idxT, const double* D, int64_t n,
                          int64_t n_w, int k, int kp1, double ns, double G, double B, double eps,
                          double* W_out, double* g_out, double* partials, double* out4,
                          void* stream);
/* The same with out4 updated in place and vals[2] = {out4[0] on entry (the previous pass's H),
 * the new KL}: the off-policy graph iteration's two control scalars (device_loop.py). */
int mepol_entropy_forward_emit(const double* w, const int32_t* idxT, const double* D, int64_t n,
                               int64_t n_w, int k, int kp1, double ns, double G, double B,
                               double eps, double* W_out, double* g_out, double* partials,
                               double* out4, double* vals, void* stream);
/* Sharded off-policy iteration (mepol_amd/parallel.py), one launch each: the all-gathered
 * per-rank [u (n) | trajectory sums (nt)] blocks normalised into w_glob [world n] (U = the sum of
 * all world * nt trajectory sums in one fixed order, the same on every rank), and the replay's
 * control scalars from the all-gathered raw sums (at offset off of each rank's block of `stride`
 * doubles): vals = {B - sums_cur[0], sum_kl / n_global}, then sums_cur = the sums. */
int mepol_iw_normalize_gathered(const double* xu_all, int world, int64_t n, int nt,
                                double* w_glob, void* stream);
int mepol_sharded_emit(const double* x_all, int world, int64_t stride, int64_t off, double B,
                       int64_t n_global, double* sums_cur, double* vals, void* stream);

/* ---- entropy gradient (the autograd of policy_update's loss.backward(), mepol.py:278) ----
 * CSR transpose of the first k rows of idxT ([>=k, nq]) for owned ids [col_offset, +ncand):
 * csr_off [ncand+1], csr_rows [nq*k] (query rows row_offset + i, stable order). */
int mepol_csr_workspace_size(int64_t nq, int k, int64_t ncand, size_t* bytes);
int mepol_csr_build(const int32_t* idxT, int64_t nq, int k, int64_t col_offset, int64_t ncand,
                    int64_t row_offset, int32_t* csr_off, int32_t* csr_rows, void* workspace,
                    size_t workspace_bytes, void* stream);
/* gamma_j = sum_{i in CSR(j)} g_i ; partials[b] = block sums of gamma_j w_j: partials holds
 * mepol_entropy_gamma_partials_size(n_own) doubles = min(ceil(8 n_own / 256), 2048) (8 lanes
 * per particle since ABI 4, grid-stride beyond). */
int mepol_entropy_gamma_partials_size(int64_t n_own);
int mepol_entropy_gamma(const double* g, const double* w_own, const int32_t* csr_off,
                        const int32_t* csr_rows, int64_t n_own, double* gamma_out,
                        double* partials, void* stream);
/* grad_logp[n, s] = grad_H * sum_{t>=s} (gamma_{n,t} - S) w_{n,t},  S = sum(partials) or *S_ext. */
int mepol_entropy_reverse_scan(const double* gamma, const double* w, const double* partials,
                               int64_t nparts, const double* S_ext, const int64_t* traj_offsets,
                               int64_t num_traj, int64_t T_stride, const double* grad_H,
                               double* grad_logp, void* stream);

/* Whole rollout of collect_particles (mepol.py:70-111, one call for all T steps) for the
 * reference's 2-hidden-layer ReLU policy on a 2-feature env: one or ceil(h1/64) workgroups per
 * trajectory (see mepol_rollout_mlp_workspace_size).
 * env_id 0 = MountainCar (init64 [n,2] f64), 1 = GridWorld (init32 [n,2] f32, a_dim = 2).
 * W1 [h0,2], b1 [h0], W2t = W2^T [h0,h1], b2 [h1], Wm [a_dim,h1], bm, log_std [a_dim];
 * noise [T,n,a_dim] f64 (a = mean + noise * exp(log_std), policy.py:59).  Writes states_rec
 * [n,T+1,2] f32, actions_rec [n,T,a_dim] f32, visited [n,T,2] f64 (nullable: the env state after
 * each step, for the heatmap) and final_state [n,2] f64 (nullable).  h0, h1 <= 512, a_dim <= 8. */
int mepol_rollout_mlp(int env_id, const double* W1, const double* b1, int h0, const double* W2t,
                      const double* b2, int h1, const double* Wm, const double* bm,
                      const double* log_std, int a_dim, const double* init64, const float* init32,
                      const double* noise, int64_t n, int64_t T, float* states_rec,
                      float* actions_rec, double* visited, double* final_state, void* workspace,
                      size_t workspace_bytes, void* stream);
/* Scratch for mepol_rollout_mlp's multi-workgroup form (ceil(h1/64) workgroups per trajectory,
 * each holding its 64 columns of W2^T in LDS; used when n * ceil(h1/64) fits the CUs and
 * h0 <= 306): one 8-byte mail word per (trajectory, step, part, action).  Word 0 of the
 * workspace is a device int32 error flag: 1 = the workgroups of a trajectory could not all run
 * at once (results invalid; the caller raises).  A null or short workspace selects the
 * one-workgroup-per-trajectory form. */
int mepol_rollout_mlp_workspace_size(int64_t n, int64_t T, int h0, int h1, int a_dim,
                                     size_t* bytes);
/* Which form mepol_rollout_mlp takes for this shape (given a sufficient workspace): workgroups
 * per trajectory, and k_chunks = the number of k-ranges the second layer's sum is split into
 * (1: one fma chain over all h0 rows; 4: four chains of ceil(h0/4) rows added in order), i.e.
 * the summation order of oracle/native/rollout_kordered.c the results match bit for bit. */
int mepol_rollout_mlp_plan_info(int64_t n, int h0, int h1, int a_dim, int* workgroups_per_traj,
                                int* k_chunks);

/* ---- policy MLP (GaussianPolicy, src/policy.py:16-51) for the large-batch passes -----------
 * Gaussian head: mean layer + log-probability with the last hidden layer's bias and ReLU folded
 * in.  z [n, hidden] is the last hidden layer's PRE-activation WITHOUT its bias bz (nullable);
 * Wm [a_dim, hidden], bm/log_std [a_dim]; act [n, a_dim].  Forward writes mu [n, a_dim] and
 * logp [n].  Backward (grad_logp [n]) writes dz [n, hidden] (nullable), dWm, dbm, dlog_std and
 * dbz [hidden] (nullable).  Limits: hidden <= 512, a_dim <= 32. */
int mepol_head_forward(const double* z, int64_t n, int hidden, const double* bz, const double* Wm,
                       const double* bm, const double* log_std, const double* act, int a_dim,
                       double* mu_out, double* logp_out, void* stream);
int mepol_head_workspace_size(int64_t n, int hidden, int a_dim, size_t* bytes);
int mepol_head_backward(const double* grad_logp, const double* z, int64_t n, int hidden,
                        const double* bz, const double* Wm, const double* log_std,
                        const double* act, const double* mu, int a_dim, double* dz, double* dWm,
                        double* dbm, double* dlog_std, double* dbz, void* workspace,
                        size_t workspace_bytes, void* stream);
/* mepol_head_backward in two launches on possibly different streams: phase 1 = the row kernel
 * (dz and the per-block records in the workspace), phase 2 = the fixed-order reduces of those
 * records into dWm, dbm, dlog_std, dbz (the caller orders phase 2 after phase 1 and keeps the
 * workspace until phase 2 ran).  Same arguments and the same bits as mepol_head_backward
 * (ABI 4; the off-policy iteration runs phase 2 beside the dW2 / dh1 GEMMs). */
int mepol_head_backward_phase(const double* grad_logp, const double* z, int64_t n, int hidden,
                              const double* bz, const double* Wm, const double* log_std,
                              const double* act, const double* mu, int a_dim, double* dz,
                              double* dWm, double* dbm, double* dlog_std, double* dbz,
                              void* workspace, size_t workspace_bytes, int phase, void* stream);
/* Input layer h = relu(x W^T + b): x [n, in] (in <= 64), W [out, in], b [out], h [n, out];
 * backward from dh = dL/dh and h: dW [out, in], db [out] (nullable). */
int mepol_layer_forward(const double* x, int64_t n, int in_features, const double* W,
                        const double* b, int out_features, double* h_out, void* stream);
int mepol_layer_workspace_size(int64_t n, int in_features, int out_features, size_t* bytes);
int mepol_layer_backward(const double* dh, const double* h, const double* x, int64_t n,
                         int in_features, int out_features, double* dW, double* db,
                         void* workspace, size_t workspace_bytes, void* stream);

/* Fused policy forward for the large-batch passes (GaussianPolicy.get_log_p, src/policy.py:21-51,
 * net = Linear(nf,h0) ReLU Linear(h0,h1) ReLU, mean = Linear(h1,a)): h1 = relu(x W1^T + b1)
 * [n, h0], z2 = h1 W2^T [n, h1] (pre-bias, as the head kernels take it), mu [n, a] and logp [n]
 * in one kernel.  in_features <= 64, hidden1 <= 320; W2 16-byte aligned. */
int mepol_policy_forward(const double* x, int64_t n, int in_features, const double* W1,
                         const double* b1, int hidden0, const double* W2, const double* b2,
                         int hidden1, const double* Wm, const double* bm, const double* log_std,
                         const double* actions, int action_dim, double* h1_out, double* z2_out,
                         double* mu_out, double* logp_out, void* stream);

/* mepol_policy_forward plus relu'(h1) as bits: h1_mask_out [n, ceil(hidden0 / 16)] uint16,
 * bit b of word w of row r = (h1[r][16 w + b] > 0), for mepol_dh1_layer1_backward_masked. */
int mepol_policy_forward_masked(const double* x, int64_t n, int in_features, const double* W1,
                                const double* b1, int hidden0, const double* W2, const double* b2,
                                int hidden1, const double* Wm, const double* bm,
                                const double* log_std, const double* actions, int action_dim,
                                double* h1_out, double* z2_out, double* mu_out, double* logp_out,
                                uint16_t* h1_mask_out, void* stream);

/* Backward of the first layer fused into the dh1 GEMM: dW1 [h0, in] and db1 [h0] (nullable) of
 * h1 = relu(x W1^T + b1) from dz2 [n, k] and W2t = W2^T [h0, k] (dh1 = dz2 W2 stays on chip,
 * masked by h1 > 0 from the forward's h1 [n, h0]).  k even, in_features <= 63, dz2 and W2t
 * 16-byte aligned; workspace from mepol_dh1_layer1_workspace_size.  Replaces the dh1
 * torch.mm + threshold_backward + dW1/db1 reductions of loss.backward() (mepol.py:278). */
int mepol_dh1_layer1_workspace_size(int64_t n, int hidden0, int in_features, size_t* bytes);
int mepol_dh1_layer1_backward(const double* dz2, int64_t n, int k, const double* W2t, int hidden0,
                              const double* h1, const double* x, int in_features, double* dW1,
                              double* db1, void* workspace, size_t workspace_bytes,
                              void* stream);
/* The same with relu'(h1) from the forward's bit mask (mepol_policy_forward_masked) instead of
 * the f64 h1 values: identical results, 1/64 of the epilogue's operand bytes. */
int mepol_dh1_layer1_backward_masked(const double* dz2, int64_t n, int k, const double* W2t,
                                     int hidden0, const uint16_t* h1_mask, const double* x,
                                     int in_features, double* dW1, double* db1, void* workspace,
                                     size_t workspace_bytes, void* stream);
/* The masked form with the second Linear's weight as stored, W2 [k][hidden0] (hidden0 even,
 * 16-B aligned), instead of W2^T: the kernel transposes its k-tiles on the way into LDS, so the
 * caller needs no W2^T copy per optimizer step (ABI 4).  Identical results. */
int mepol_dh1_layer1_backward_w2(const double* dz2, int64_t n, int k, const double* W2,
                                 int hidden0, const uint16_t* h1_mask, const double* x,
                                 int in_features, double* dW1, double* db1, void* workspace,
                                 size_t workspace_bytes, void* stream);

/* Weight gradient of a linear layer over a tall batch: dW [out, in] = dy^T x with dy [n, out]
 * and x [n, in] row-major f64 (the policy's dW2 = dz2^T h1, K = n), split-K on the f64 matrix
 * cores and summed over the K-slices in a fixed order; workspace from
 * mepol_weight_grad_workspace_size.  Replaces the weight gradient of the second Linear in
 * loss.backward() (src/policy.py:21-26, mepol.py:278). */
int mepol_weight_grad_workspace_size(int64_t n, int out_features, int in_features, size_t* bytes);
int mepol_weight_grad(const double* dy, int64_t n, int out_features, const double* x,
                      int in_features, double* dW, void* workspace, size_t workspace_bytes,
                      void* stream);

/* Hidden layer on the f64 matrix cores: C = act(A B^T + bias), A [n, k] (row stride lda),
 * B [m, k] (ldb), bias [m] (nullable), C [n, m] (ldc); act = ReLU when relu != 0.  k, lda, ldb
 * even and A, B 16-byte aligned.  variant 0 = default tiling.  Replaces the torch.mm /
 * nn.Linear GEMMs of GaussianPolicy.net (src/policy.py:21-26) in the large-batch passes. */
int mepol_gemm_nt(const double* A, int64_t n, int k, int64_t lda, const double* B, int m,
                  int64_t ldb, const double* bias, int relu, double* C, int64_t ldc, int variant,
                  void* stream);

/* ---- environments -------------------------------------------------------------------------
 * Replace MountainCarContinuous.step (src/envs/mountain_car_wall.py:13-45) and
 * GridWorldContinuous.step (src/envs/gridworld_continuous.py:128-154), batched. */
int mepol_step_mountaincar(double* state, const double* action, int64_t n, int64_t action_stride,
                           void* stream);
int mepol_step_gridworld(float* state, const double* action, int64_t n, void* stream);
/* One step of collect_particles (mepol.py:81-90) for n trajectories: a = mean + noise*exp(log_std),
 * record s_{t+1}/a_t as f32, advance the env. env_id 0 = MountainCar, 1 = GridWorld. */
int mepol_rollout_step(int env_id, double* env_f64, float* env_f32, const double* mean,
                       const double* noise, const double* log_std, int64_t n, int a_dim, int64_t t,
                       int64_t T, float* states_rec, float* actions_rec, double* policy_in,
                       void* stream);

/* ---- Optimizer step of policy_update (mepol.py:280, optimizer.step()) ------------------------
 * Replaces torch.optim.Adam(lr).step() (kind 0) / torch.optim.RMSprop(lr).step() (kind 1) as
 * constructed at mepol.py:308-311, over n_tensors (<= 8) f64 parameter tensors in one launch.
 * exp_avg (Adam only) / exp_avg_sq (Adam; RMSprop square_avg) are updated in place.
 * scalars is DEVICE memory: Adam {enable, lr/bias_correction1, sqrt(bias_correction2), beta1,
 * beta2, eps}; RMSprop {enable, lr, alpha, eps}.  enable == 0 makes the call a no-op. */
int mepol_optim_step(int kind, int n_tensors, double* const* params, const double* const* grads,
                     double* const* exp_avg, double* const* exp_avg_sq, const int64_t* sizes,
                     const double* scalars, void* stream);
/* mepol_optim_step that also writes each tensor's values from before the update into
 * params_snap / exp_avg_snap / exp_avg_sq_snap (arrays of n_tensors device pointers, each array
 * may be NULL): the device iteration's shadow of the last accepted theta and its optimizer-moment
 * snapshot (algorithms/device_loop.py, mepol.py:441-456 semantics). */
int mepol_optim_step_snapshot(int kind, int n_tensors, double* const* params,
                              const double* const* grads, double* const* exp_avg,
                              double* const* exp_avg_sq, const int64_t* sizes,
                              const double* scalars, double* const* params_snap,
                              double* const* exp_avg_snap, double* const* exp_avg_sq_snap,
                              void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MEPOL_AMD_H */
