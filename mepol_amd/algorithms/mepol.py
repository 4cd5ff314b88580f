"""MEPOL hot path on MI355X: drop-in for src/algorithms/mepol.py of the reference.

Same function names, argument order/meaning and return types as the reference
(src/algorithms/mepol.py), with the particle batch resident in HBM:

  collect_particles(env, policy, num_traj, traj_len, state_filter)            :70-111
  compute_importance_weights(behavioral, target, states, actions, nt, rtl)   :114-139
  compute_entropy(..., distances, indices, k, G, B, ns, eps)                  :142-154
  compute_kl(..., distances, indices, k, eps)                                 :157-174
  collect_particles_and_compute_knn(env, policy, nt, T, state_filter, k, W)   :177-202
  policy_update(optimizer, behavioral, target, ..., k, G, B, ns, eps)         :268-281
  mepol(env, env_name, state_filter, create_policy, k, kl_threshold, ...)     :284-545

Differences a caller can observe (all documented in DESIGN.md):
  * tensors returned by collect_particles_and_compute_knn live on the GPU (the reference's
    "#todo: any target device", mepol.py:194); collect_particles still returns numpy;
  * k-NN ties are broken by the smaller index (sklearn's order is implementation-defined);
  * rollout noise comes from torch's device generator, so trajectories are not the CPU
    reference's random stream (dynamics are; see tests/test_gpu_envs.py).
"""
import atexit
import math
import os
import time
import weakref

import numpy as np
import scipy.special
import torch
import torch.nn as nn

from .. import ops
from ..envs.wrappers import unwrap
from . import particles as P

float_type = torch.float64
int_type = torch.int64


# ---------------------------------------------------------------------------------------------
# Rollout
# ---------------------------------------------------------------------------------------------
def _batched_kind(env):
    return getattr(type(unwrap(env)), "batched_kind", None)


class _RolloutGraph:
    """The T-step rollout of a HIP-stepped env as one replayed HIP graph.

    Each step is the policy MLP (a few small GEMM / ReLU launches) plus the fused
    rollout_step kernel: at MEPOL's batch sizes (tens to hundreds of trajectories) the loop is
    launch-bound (~65 us per step eager).  Captured once per (policy, env, shape) into static
    buffers -- initial states, the pre-drawn noise [T, n, a], the recorded states / actions --
    and replayed every epoch; the policy's parameters are read in place, so load_state_dict
    between epochs needs no re-capture."""

    def __init__(self, policy, env_id, init, T, a_dim, nf):
        dev = init.device
        n = init.shape[0]
        self.key = (env_id, n, T, a_dim, nf, tuple(p.data_ptr() for p in policy.parameters()))
        self.init = init.clone()
        self.noise = torch.zeros((T, n, a_dim), dtype=torch.float64, device=dev)
        self.states = torch.zeros((n, T + 1, nf), dtype=torch.float32, device=dev)
        self.actions = torch.zeros((n, T, a_dim), dtype=torch.float32, device=dev)
        self.env = torch.empty_like(init)
        self.policy_in = torch.empty((n, nf), dtype=torch.float64, device=dev)
        self.log_std = policy.log_std.detach()
        # weak: the cache entry is keyed by the policy and must not keep it alive
        self.env_id, self.T, self._policy = env_id, T, weakref.ref(policy)
        # warm-up (library handles, workspaces) outside the capture, then capture
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            self._body(1)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side, capture_error_mode="thread_local"):
            self._body(T)
        torch.cuda.current_stream().wait_stream(side)

    def _body(self, steps):
        self.env.copy_(self.init)
        self.policy_in.copy_(self.init)
        self.states[:, 0].copy_(self.init)
        e64 = self.env if self.env_id == 0 else None
        e32 = self.env if self.env_id == 1 else None
        for t in range(steps):
            mean = self._policy().mean_action(self.policy_in).contiguous()
            ops.rollout_step(self.env_id, e64, e32, mean, self.noise[t], self.log_std, t, self.T,
                             self.states, self.actions, self.policy_in)

    def run(self, init, noise):
        self.init.copy_(init)
        self.noise.copy_(noise)
        self.graph.replay()
        return self.states.clone(), self.actions.clone()


_ROLLOUT_GRAPHS = weakref.WeakKeyDictionary()  # policy -> {key: _RolloutGraph}


@atexit.register
def _release_graphs_at_exit():
    """Drop every captured graph (rollout, off-policy loop, sharded loop) while the HIP runtime
    is still up: left to interpreter teardown they can be destroyed after it (a segfault at exit
    was seen under rocprofv3)."""
    try:
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 - best effort at exit
        pass
    _ROLLOUT_GRAPHS.clear()
    import sys

    dl = sys.modules.get("mepol_amd.algorithms.device_loop")
    if dl is not None:
        for it in list(dl._CACHE.values()):
            it.release()
        dl._CACHE.clear()
    par = sys.modules.get("mepol_amd.parallel")
    if par is not None:
        par.release_graphs()


def _rollout_graph(policy, env_id, init, T, a_dim, nf):
    if os.environ.get("MEPOL_ROLLOUT_GRAPH", "1") == "0" or not policy.log_std.is_contiguous():
        return None
    key = (env_id, init.shape[0], T, a_dim, nf, tuple(p.data_ptr() for p in policy.parameters()))
    per = _ROLLOUT_GRAPHS.setdefault(policy, {})
    g = per.get(key)
    if g is None:
        if len(per) >= 4:  # bounded: the epoch and full-entropy shapes of a run
            per.clear()
        g = per[key] = _RolloutGraph(policy, env_id, init, T, a_dim, nf)
    return g


def _rollout_mlp_layers(policy, nf, a_dim):
    """((W1, b1), (W2, b2)) when the policy is the reference's nf = 2 -> [h0, h1] -> a ReLU MLP in
    f64 that the one-launch rollout kernel covers (h <= 512, a <= 8); else None."""
    if os.environ.get("MEPOL_ROLLOUT_FUSED", "1") == "0" or nf != 2 or a_dim > 8:
        return None
    if getattr(policy, "activation", None) is not nn.ReLU:
        return None
    layers = [m for m in policy.net if isinstance(m, nn.Linear)]
    if len(layers) != 2 or any(m.weight.dtype != torch.float64 for m in layers):
        return None
    if layers[0].in_features != 2 or max(m.out_features for m in layers) > 512:
        return None
    return tuple((m.weight.detach(), m.bias.detach()) for m in layers)


def collect_particles_device(env, policy, num_traj, traj_len, state_filter, generator=None,
                             visited=None, shard=None):
    """Rollout of num_traj trajectories of traj_len steps, batched on the policy's device.

    Returns device tensors: states f32 [nt, T+1, nf], actions f32 [nt, T, a], real lengths
    int32 [nt, 1], next_states f32 [N, ns] (particle p = n*T + t <-> s_{n, t+1}, mepol.py:98-109).
    MountainCar / GridWorld step in a HIP kernel (one fused launch per step after the MLP);
    any other env is stepped on the host in lockstep with one batched policy call per step.
    `visited` (optional, f64 [nt, T, nf]) receives the env's own state after every step (f64
    MountainCar state / GridWorld f32 state, not the f32 particle copy), for the heatmap.

    shard=(rank, world): roll out only trajectories [rank nt/world, (rank+1) nt/world) of the
    num_traj-trajectory batch.  The initial states and the action noise of ALL trajectories are
    drawn up front ([T, nt, a] f64, one draw), so a trajectory's randomness does not depend on
    how the batch is split: the shards of `world` ranks concatenate to the one-rank rollout (the
    reference's loky workers instead start from copies of one RNG state).
    """
    dev = policy.device
    if dev.type != "cuda":
        raise RuntimeError("collect_particles_device needs the policy on a ROCm device")
    base = unwrap(env)
    kind = _batched_kind(env)
    nf = env.num_features
    a_dim = env.action_space.shape[0]
    T = int(traj_len)
    rank, world = shard if shard is not None else (0, 1)
    if num_traj % world:
        raise ValueError(f"{num_traj} trajectories do not split over {world} ranks")
    total = num_traj
    num_traj = total // world
    lo, hi = rank * num_traj, (rank + 1) * num_traj
    states = torch.zeros((num_traj, T + 1, nf), dtype=torch.float32, device=dev)
    actions = torch.zeros((num_traj, T, a_dim), dtype=torch.float32, device=dev)
    with torch.no_grad():
        if kind in ("mountaincar", "gridworld"):
            env_id = 0 if kind == "mountaincar" else 1
            init = base.reset_batch_torch(total, dev, generator)[lo:hi]
            noise_all = torch.randn((T, total, a_dim), dtype=torch.float64, device=dev,
                                    generator=generator)
            lin = _rollout_mlp_layers(policy, nf, a_dim)
            if lin is not None:  # all T steps in one launch (csrc/envs.hip rollout_mlp_kernel)
                (W1, b1), (W2, b2) = lin
                ops.rollout_mlp(env_id, W1, b1, W2, b2, policy.mean.weight.detach(),
                                policy.mean.bias.detach(), policy.log_std.detach(), init,
                                noise_all[:, lo:hi], states, actions, visited)
                rtl = torch.full((num_traj, 1), T, dtype=torch.int32, device=dev)
                next_states = states[:, 1:, :].reshape(-1, nf)
                if state_filter is not None:
                    next_states = next_states[:, list(state_filter)]
                return states, actions, rtl, next_states.contiguous()
            graph = _rollout_graph(policy, env_id, init, T, a_dim, nf) if visited is None else None
            if graph is not None:
                states, actions = graph.run(init, noise_all[:, lo:hi])
                rtl = torch.full((num_traj, 1), T, dtype=torch.int32, device=dev)
                next_states = states[:, 1:, :].reshape(-1, nf)
                if state_filter is not None:
                    next_states = next_states[:, list(state_filter)]
                return states, actions, rtl, next_states.contiguous()
            env64 = init.clone() if env_id == 0 else None
            env32 = init.clone() if env_id == 1 else None
            policy_in = init.to(torch.float64).contiguous()
            states[:, 0] = init.to(torch.float32)
            log_std = policy.log_std.detach().contiguous()
            for t in range(T):
                mean = policy.mean_action(policy_in).contiguous()
                noise = noise_all[t, lo:hi]
                ops.rollout_step(env_id, env64, env32, mean, noise, log_std, t, T, states, actions,
                                 policy_in)
                if visited is not None:
                    visited[:, t].copy_(policy_in)
        else:
            if world > 1:
                raise NotImplementedError("sharded rollouts need a batched (HIP-stepped) env")
            envs = [env] + [_clone_env(env) for _ in range(num_traj - 1)]
            s = np.stack([e.reset() for e in envs])
            states[:, 0] = torch.as_tensor(s, dtype=torch.float32, device=dev)
            for t in range(T):
                x = torch.as_tensor(s, dtype=torch.float64, device=dev)
                _, a = policy(x)
                actions[:, t] = a.to(torch.float32)
                a_np = a.cpu().numpy()
                s = np.stack([e.step(a_np[i])[0] for i, e in enumerate(envs)])
                states[:, t + 1] = torch.as_tensor(s, dtype=torch.float32, device=dev)
                if visited is not None:
                    visited[:, t] = torch.as_tensor(s, dtype=torch.float64, device=dev)
    rtl = torch.full((num_traj, 1), T, dtype=torch.int32, device=dev)
    next_states = states[:, 1:, :].reshape(-1, nf)
    if state_filter is not None:
        next_states = next_states[:, list(state_filter)]
    return states, actions, rtl, next_states.contiguous()


def get_heatmap(env, policy, discretizer, num_episodes, num_steps, cmap, interp, labels):
    """State-visitation heatmap of the policy (mepol.py:19-67), all episodes in one rollout.

    The reference runs num_episodes episodes of num_steps steps one after another and stops an
    episode on `done`; every MEPOL env is wrapped in ErgodicEnv (done is always False), so each
    episode is exactly num_steps steps and the episodes are the trajectories of one batched
    collect_particles_device call.  The visited states are recorded in f64 and binned on the
    device (Discretizer.visitation_stats, np.digitize semantics).  Returns
    (average_state_dist ndarray [bins], average_entropy float, figure; None without matplotlib).
    """
    nf = env.num_features
    visited = torch.empty((num_episodes, num_steps, nf), dtype=torch.float64,
                          device=policy.device)
    collect_particles_device(env, policy, num_episodes, num_steps, None, visited=visited)
    dist, ent = discretizer.visitation_stats(visited)
    average_state_dist = dist.cpu().numpy()
    image = _heatmap_figure(average_state_dist, discretizer.bins_sizes, cmap, interp, labels)
    return average_state_dist, float(ent), image


def _heatmap_figure(average_state_dist, bins_sizes, cmap, interp, labels):
    """The reference's figure (mepol.py:49-65): log-probability image (2-D) or bar chart."""
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except Exception:
        return None
    plt.close()
    fig = plt.figure()
    plt.xticks([])
    plt.yticks([])
    if labels is not None:
        plt.xlabel(labels[0])
        plt.ylabel(labels[1])
    if average_state_dist.ndim == 2:
        log_p = np.ma.log(average_state_dist)
        flat = log_p.ravel()
        lo = np.min(flat)
        rest = flat[flat != lo]
        if rest.count() > 0:
            flat[np.argmin(flat)] = np.min(rest)
        plt.imshow(log_p.filled(lo), interpolation=interp, cmap=cmap)
    else:
        plt.bar(list(range(bins_sizes[0])), average_state_dist)
    return fig


def _clone_env(env):
    import copy

    return copy.deepcopy(env)


def collect_particles(env, policy, num_traj, traj_len, state_filter):
    """Reference signature (mepol.py:70-111): numpy f32 states/actions/next_states, i32 lengths."""
    s, a, r, ns = collect_particles_device(env, policy, num_traj, traj_len, state_filter)
    return s.cpu().numpy(), a.cpu().numpy(), r.cpu().numpy(), ns.cpu().numpy()


def collect_particles_and_compute_knn(env, behavioral_policy, num_traj, traj_len, state_filter, k,
                                      num_workers):
    """Rollout + exact k-NN (mepol.py:177-202); tensors stay on the GPU.

    num_workers keeps the reference's divisibility contract (mepol.py:179); the whole batch is
    rolled out by the GPU, so no worker processes are spawned.
    """
    assert num_traj % num_workers == 0, "Please provide a number of trajectories " \
                                        "that can be equally split among workers"
    s32, a32, rtl32, ns32 = collect_particles_device(env, behavioral_policy, num_traj, traj_len,
                                                     state_filter)
    # host copy of the lengths before the k-NN is queued: read after it, it would make the host
    # wait for the whole k-NN and leave the GPU idle while the batch is set up
    lens_host = rtl32.reshape(-1).to(torch.int64).cpu()
    # the k-NN's input check is read once the work behind it is queued (mepol_knn_deferred)
    D, I, I32T, check = ops.knn(ns32, k + 1, defer_check=True)
    states = s32.to(float_type)
    actions = a32.to(float_type)
    next_states = ns32.to(float_type)
    real_traj_lengths = rtl32.to(int_type)
    batch = P.ParticleBatch(states, actions, real_traj_lengths, D, I, idx32T=I32T,
                            lengths=lens_host)
    _register_checked(I, batch, k, check)
    return states, actions, real_traj_lengths, next_states, D, I


def make_particle_batch(states, actions, real_traj_lengths, next_states_f32, k,
                        knn_events=None):
    """Register a batch built from externally produced particles (e.g. a MuJoCo rollout or a
    synthetic benchmark batch): runs the GPU k-NN and returns the reference's 6-tuple.
    knn_events: optional (start, end) CUDA events recorded around the k-NN call alone."""
    lens_host = real_traj_lengths.reshape(-1).to(torch.int64).cpu()  # before the k-NN: see above
    if knn_events is not None:
        knn_events[0].record()
    D, I, I32T, check = ops.knn(next_states_f32, k + 1, defer_check=True)
    if knn_events is not None:
        knn_events[1].record()
    batch = P.ParticleBatch(states, actions, real_traj_lengths, D, I, idx32T=I32T,
                            lengths=lens_host)
    _register_checked(I, batch, k, check)
    return states, actions, real_traj_lengths, next_states_f32.to(float_type), D, I


def _register_checked(I, batch, k, check):
    """Register the epoch's batch and queue its CSR build (the GPU builds it while the host
    sets up the off-policy loop), then read the k-NN's deferred input check: a rejected input
    (sklearn's check_array ValueError, as kneighbors raises it) leaves no batch registered."""
    P.register(I, batch)
    batch.csr(k)
    try:
        check.raise_if_invalid()
    except ValueError:
        P.unregister(I)
        raise


# ---------------------------------------------------------------------------------------------
# Importance weights / entropy / KL
# ---------------------------------------------------------------------------------------------
class _IWFunction(torch.autograd.Function):
    """w = normalize(exp(segmented cumsum(logp_t - logp_b))) with its exact backward."""

    @staticmethod
    def forward(ctx, logp_t, logp_b, batch):
        _, _, w, _ = ops.iw_forward(logp_t.detach(), logp_b.detach(), batch.offsets, batch.N)
        ctx.batch = batch
        ctx.save_for_backward(w)
        return w

    @staticmethod
    def backward(ctx, grad_w):
        (w,) = ctx.saved_tensors
        b = ctx.batch
        grad_w = grad_w.contiguous()
        S = torch.dot(grad_w, w).reshape(())
        one = torch.ones((), dtype=torch.float64, device=w.device)
        grad = ops.entropy_reverse_scan(grad_w, w, S, 0, b.offsets, b.num_traj, b.T, one, S_ext=S)
        return grad, None, None


class _EntropyFunction(torch.autograd.Function):
    """H(logp_t) of compute_entropy, fused with compute_kl's statistic (one forward).

    forward: IW scan + normalise + gather/volume/log terms (HIP); saves w and dH/dW.
    backward: CSR gather of dH/dW -> gamma, S = <gamma, w>, segmented reverse scan (HIP);
    the result is dH/dlogp_t, which torch autograd pushes through the MLP.
    """

    @staticmethod
    def forward(ctx, logp_t, logp_b, batch, k, G, B, ns, eps):
        _, _, w, _ = ops.iw_forward(logp_t.detach(), logp_b.detach(), batch.offsets, batch.N)
        out4, _, g = ops.entropy_forward(w, batch.idx32T, batch.D, k, ns, G, B, eps)
        ctx.batch, ctx.k = batch, k
        ctx.save_for_backward(w, g)
        ctx.out4 = out4
        ctx.mark_non_differentiable(out4)
        return out4[0].clone(), out4

    @staticmethod
    def backward(ctx, grad_H, _grad_out4):
        w, g = ctx.saved_tensors
        b = ctx.batch
        off, rows = b.csr(ctx.k)
        gamma, partials, nparts = ops.entropy_gamma(g, w, off, rows)
        gH = grad_H.reshape(()).to(torch.float64).contiguous()
        grad = ops.entropy_reverse_scan(gamma, w, partials, nparts, b.offsets, b.num_traj, b.T, gH)
        return grad, None, None, None, None, None, None, None


def _logps(batch, behavioral_policy, target_policy):
    logp_b = batch.behavioral_logp(behavioral_policy)
    if target_policy is behavioral_policy:
        return logp_b, logp_b
    if torch.is_grad_enabled():
        stashed = batch.take_logp(target_policy)
        if stashed is not None:
            return stashed, logp_b
    return batch.logp(target_policy), logp_b


def compute_importance_weights(behavioral_policy, target_policy, states, actions, num_traj,
                               real_traj_lengths):
    """Normalised per-particle importance weights w [N] f64 (mepol.py:114-139), differentiable
    w.r.t. the target policy's parameters."""
    batch = P.ParticleBatch(states, actions, real_traj_lengths,
                            torch.zeros((1, 2), dtype=torch.float64),
                            torch.zeros((1, 2), dtype=torch.int64))
    logp_t, logp_b = _logps(batch, behavioral_policy, target_policy)
    return _IWFunction.apply(logp_t, logp_b, batch)


def _entropy_device(behavioral_policy, target_policy, states, actions, num_traj,
                    real_traj_lengths, distances, indices, k, G, B, ns, eps):
    """compute_entropy's estimate left on the device (no host synchronisation)."""
    batch = P.lookup(states, actions, real_traj_lengths, distances, indices)
    logp_t, logp_b = _logps(batch, behavioral_policy, target_policy)
    H, _ = _EntropyFunction.apply(logp_t, logp_b, batch, k, G, B, ns, eps)
    return H


def compute_entropy(behavioral_policy, target_policy, states, actions, num_traj, real_traj_lengths,
                    distances, indices, k, G, B, ns, eps):
    """KL (Kozachenko-Leonenko) entropy estimate, 0-d f64 (mepol.py:142-154).

    Returned on the host, as the reference's CPU computation returns it: its caller reads it
    with .numpy() (mepol.py:367-368, 497-498).  The copy is differentiable, so
    ``(-compute_entropy(...)).backward()`` reaches the target policy's parameters on the GPU."""
    return _entropy_device(behavioral_policy, target_policy, states, actions, num_traj,
                           real_traj_lengths, distances, indices, k, G, B, ns, eps).cpu()


def compute_kl_deferred(behavioral_policy, target_policy, states, actions, num_traj,
                        real_traj_lengths, distances, indices, k, eps):
    """compute_kl with the numeric-error flag left on the device (a 0-d bool tensor), so the
    off-policy loop reads every control scalar of an iteration with one synchronisation."""
    batch = P.lookup(states, actions, real_traj_lengths, distances, indices)
    logp_b = batch.behavioral_logp(behavioral_policy)
    if target_policy is behavioral_policy:
        logp_t = logp_b
    elif torch.is_grad_enabled() and any(p.requires_grad for p in target_policy.parameters()):
        logp_t = batch.logp(target_policy)
        batch.stash_logp(target_policy, logp_t)
    else:
        with torch.no_grad():
            logp_t = batch.logp(target_policy)
    with torch.no_grad():
        _, _, w, _ = ops.iw_forward(logp_t.detach(), logp_b, batch.offsets, batch.N)
        out4, _, _ = ops.entropy_forward(w, batch.idx32T, batch.D, k, 1.0, 1.0, 0.0, eps)
    kl = out4[1].clone()
    return torch.clamp_min(kl, 0.0), ~torch.isfinite(kl)


def compute_kl(behavioral_policy, target_policy, states, actions, num_traj, real_traj_lengths,
               distances, indices, k, eps):
    """k-NN KL(behavioral || target) estimate and its numeric-error flag (mepol.py:157-174).

    When gradients are enabled, the target policy's MLP forward is kept (with its graph) so a
    following policy_update at the same parameters reuses it instead of recomputing it; the
    returned values are those of the reference's no_grad computation.
    """
    kl, flag = compute_kl_deferred(behavioral_policy, target_policy, states, actions, num_traj,
                                   real_traj_lengths, distances, indices, k, eps)
    return kl.cpu(), bool(flag)  # host tensor, as the reference's (its caller: kl.numpy(), :439)


def policy_update_deferred(optimizer, behavioral_policy, target_policy, states, actions, num_traj,
                           traj_len, distances, indices, k, G, B, ns, eps):
    """policy_update with the numeric-error flag (taken on the loss before backward, as at
    mepol.py:274-276) left on the device as a 0-d bool tensor."""
    optimizer.zero_grad()
    loss = -_entropy_device(behavioral_policy, target_policy, states, actions, num_traj, traj_len,
                            distances, indices, k, G, B, ns, eps)
    flag = ~torch.isfinite(loss.detach())
    loss.backward()
    optimizer.step()
    return loss, flag


def policy_update(optimizer, behavioral_policy, target_policy, states, actions, num_traj, traj_len,
                  distances, indices, k, G, B, ns, eps):
    """One gradient step maximising the entropy estimate (mepol.py:268-281).

    The 5th positional argument is the real trajectory lengths, as at the reference call site
    (mepol.py:429-431).
    """
    loss, flag = policy_update_deferred(optimizer, behavioral_policy, target_policy, states,
                                        actions, num_traj, traj_len, distances, indices, k, G, B,
                                        ns, eps)
    # host tensor, as the reference's (its caller: -loss.detach().numpy(), mepol.py:432)
    return loss.detach().cpu(), bool(flag)


# ---------------------------------------------------------------------------------------------
# Logging (output formats of mepol.py:205-265)
# ---------------------------------------------------------------------------------------------
def _summary_writer(out_path):
    try:
        if out_path is None:  # non-zero ranks of a multi-rank run log nothing
            raise RuntimeError
        from torch.utils import tensorboard  # noqa: F401

        return tensorboard.SummaryWriter(out_path)
    except Exception:
        class _Null:
            def add_scalar(self, *a, **kw):
                pass

            def add_figure(self, *a, **kw):
                pass

        return _Null()


def _distributed():
    """torch.distributed when a multi-rank process group is up (mepol() then shards), else None."""
    try:
        import torch.distributed as dist
    except ImportError:  # pragma: no cover
        return None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist
    return None


def _is_rank0():
    d = _distributed()
    return d is None or d.get_rank() == 0


def log_epoch_statistics(writer, log_file, csv_file_1, csv_file_2, epoch, loss, entropy,
                         num_off_iters, execution_time, full_entropy, heatmap_image,
                         heatmap_entropy, backtrack_iters, backtrack_lr):
    writer.add_scalar("Loss", loss, global_step=epoch)
    writer.add_scalar("Entropy", entropy, global_step=epoch)
    writer.add_scalar("Execution time", execution_time, global_step=epoch)
    writer.add_scalar("Number off-policy iteration", num_off_iters, global_step=epoch)
    if full_entropy is not None:
        writer.add_scalar("Full Entropy:", full_entropy, global_step=epoch)
    # the reference keys the heatmap outputs on the figure (mepol.py:216,230,247); here on the
    # entropy, so the CSV row is kept when matplotlib is absent
    if heatmap_image is not None:
        writer.add_figure("Heatmap", heatmap_image, global_step=epoch)
    if heatmap_entropy is not None:
        writer.add_scalar("Discrete entropy", heatmap_entropy, global_step=epoch)
    rows = [["Epoch", epoch], ["Execution time (s)", f"{execution_time:.3f}"],
            ["Entropy", f"{entropy:.3f}"], ["Off-policy iters", num_off_iters]]
    if heatmap_entropy is not None:
        rows.append(["Heatmap entropy", f"{heatmap_entropy:.3f}"])
    if backtrack_iters is not None:
        rows.append(["Backtrack iters", backtrack_iters])
    try:
        from tabulate import tabulate

        grid = tabulate(rows, headers="firstrow", tablefmt="fancy_grid", numalign="right")
    except ImportError:
        grid = "\n".join(f"{a}: {b}" for a, b in rows)
    csv_file_1.write(f"{epoch},{loss},{entropy},{full_entropy},{num_off_iters},{execution_time}\n")
    csv_file_1.flush()
    if heatmap_entropy is not None and csv_file_2 is not None:
        csv_file_2.write(f"{epoch},{heatmap_entropy}\n")
        csv_file_2.flush()
    log_file.write(grid)
    log_file.flush()
    if _is_rank0():
        print(grid)


def log_off_iter_statistics(writer, csv_file_3, epoch, global_off_iter, num_off_iter, entropy, kl,
                            lr):
    csv_file_3.write(f"{epoch},{num_off_iter},{entropy},{kl},{lr}\n")
    csv_file_3.flush()
    writer.add_scalar("Off policy iter Entropy", entropy, global_step=global_off_iter)
    writer.add_scalar("Off policy iter KL", kl, global_step=global_off_iter)


def _save_policy(policy, path):
    torch.save({k: v.detach().cpu() for k, v in policy.state_dict().items()}, path)


# ---------------------------------------------------------------------------------------------
# Driver
# ---------------------------------------------------------------------------------------------
def mepol(env, env_name, state_filter, create_policy, k, kl_threshold, max_off_iters,
          use_backtracking, backtrack_coeff, max_backtrack_try, eps, learning_rate, num_traj,
          traj_len, num_epochs, optimizer, full_entropy_traj_scale, full_entropy_k, heatmap_every,
          heatmap_discretizer, heatmap_episodes, heatmap_num_steps, heatmap_cmap, heatmap_labels,
          heatmap_interp, seed, out_path, num_workers):
    """The MEPOL epoch loop (mepol.py:284-545) with the reference's control flow and outputs.

    Heatmaps (mepol.py:19-67) are computed on the device (get_heatmap) when a discretizer is
    given, at epoch 0 and every heatmap_every epochs, and logged to {env_name}-heatmap.csv.

    Multi-rank (a torch.distributed group of world > 1 is initialised, one process per GPU):
    the particle batch is sharded by trajectory -- the reference's worker split, mepol.py:179-187
    -- and every rank holds the same policies, optimizer state and control decisions
    (parallel.ShardedEpoch: RCCL all-gather of next states before the k-NN, fixed-order
    reductions per iteration).  Rank 0 writes the logs, CSVs and checkpoints.
    """
    dist = _distributed()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist is not None else (0, 1)
    if num_traj % world:
        raise ValueError(f"num_traj={num_traj} does not split over {world} ranks")
    if seed is not None:
        np.random.seed(seed)
        torch.manual_seed(seed)
        env.seed(seed)

    behavioral_policy = create_policy(is_behavioral=True)
    target_policy = create_policy()
    last_valid_target_policy = create_policy()
    target_policy.load_state_dict(behavioral_policy.state_dict())
    last_valid_target_policy.load_state_dict(behavioral_policy.state_dict())

    if optimizer == "rmsprop":
        optimizer = torch.optim.RMSprop(target_policy.parameters(), lr=learning_rate)
    elif optimizer == "adam":
        optimizer = torch.optim.Adam(target_policy.parameters(), lr=learning_rate)
    else:
        raise NotImplementedError

    def out(name, mode="w"):  # rank 0 writes the run's files; the other ranks discard
        return open(os.path.join(out_path, name) if rank == 0 else os.devnull, mode,
                    encoding="utf-8")

    writer = _summary_writer(out_path) if rank == 0 else _summary_writer(None)
    log_file = out("log_file.txt", "a")
    csv_file_1 = out(f"{env_name}.csv")
    csv_file_1.write(",".join(["epoch", "loss", "entropy", "full_entropy", "num_off_iters",
                               "execution_time"]))
    csv_file_1.write("\n")
    if heatmap_discretizer is not None:
        csv_file_2 = out(f"{env_name}-heatmap.csv")
        csv_file_2.write(",".join(["epoch", "average_entropy"]))
        csv_file_2.write("\n")
    else:
        csv_file_2 = None

    def heatmap():
        if heatmap_discretizer is None:
            return None, None
        _, h, image = get_heatmap(env, behavioral_policy, heatmap_discretizer, heatmap_episodes,
                                  heatmap_num_steps, heatmap_cmap, heatmap_interp, heatmap_labels)
        return h, image

    csv_file_3 = out(f"{env_name}_off_policy_iter.csv")
    csv_file_3.write(",".join(["epoch", "off_policy_iter", "entropy", "kl", "learning_rate"]))
    csv_file_3.write("\n")

    ns = len(state_filter) if (state_filter is not None) else env.num_features
    B = np.log(k) - scipy.special.digamma(k)
    full_B = np.log(full_entropy_k) - scipy.special.digamma(full_entropy_k)
    G = scipy.special.gamma(ns / 2 + 1)

    def collect(nt, kk):
        """The epoch's particles: the reference's 6-tuple (one rank) or a ShardedEpoch."""
        if dist is None:
            return collect_particles_and_compute_knn(env, behavioral_policy, nt, traj_len,
                                                     state_filter, kk, num_workers)
        from ..parallel import ShardedEpoch

        assert nt % num_workers == 0, "Please provide a number of trajectories " \
                                      "that can be equally split among workers"
        s32, a32, r32, ns32 = collect_particles_device(env, behavioral_policy, nt, traj_len,
                                                       state_filter, shard=(rank, world))
        ep = ShardedEpoch(s32.to(float_type), a32.to(float_type), r32.to(int_type), ns32, kk,
                          dist)
        ep.build_knn()
        return ep

    def no_grad_entropy(batch, nt, kk, BB):
        with torch.no_grad():
            if dist is not None:
                return batch.compute_entropy(behavioral_policy, behavioral_policy, kk, G, BB, ns,
                                             eps)
            st, ac, rl, _, D, I = batch
            return compute_entropy(behavioral_policy, behavioral_policy, st, ac, nt, rl, D, I, kk,
                                   G, BB, ns, eps)

    epoch = 0
    _sync()
    t0 = time.time()
    full_entropy = no_grad_entropy(collect(num_traj * full_entropy_traj_scale, full_entropy_k),
                                   num_traj * full_entropy_traj_scale, full_entropy_k, full_B)
    entropy = no_grad_entropy(collect(num_traj, k), num_traj, k, B)
    full_entropy = _np(full_entropy)
    entropy = _np(entropy)
    execution_time = time.time() - t0
    loss = -entropy
    heatmap_entropy, heatmap_image = heatmap()
    if rank == 0:
        _save_policy(behavioral_policy, os.path.join(out_path, f"{epoch}-policy"))
    log_epoch_statistics(writer=writer, log_file=log_file, csv_file_1=csv_file_1,
                         csv_file_2=csv_file_2, epoch=epoch, loss=loss, entropy=entropy,
                         execution_time=execution_time, num_off_iters=0, full_entropy=full_entropy,
                         heatmap_image=heatmap_image, heatmap_entropy=heatmap_entropy,
                         backtrack_iters=None, backtrack_lr=None)

    global_num_off_iters = 0
    original_lr = learning_rate

    while epoch < num_epochs:
        _sync()
        t0 = time.time()
        last_valid_target_policy.load_state_dict(behavioral_policy.state_dict())

        batch = collect(num_traj, k)

        def on_accept(num_off_iters, entropy, kl, lr):
            nonlocal global_num_off_iters
            global_num_off_iters += 1
            log_off_iter_statistics(writer, csv_file_3, epoch, global_num_off_iters,
                                    num_off_iters - 1, entropy, kl, lr)

        lr0 = original_lr if use_backtracking else learning_rate
        if dist is not None:
            res = batch.off_policy_optimization(
                optimizer, behavioral_policy, target_policy, last_valid_target_policy, G, B, ns,
                eps, kl_threshold, max_off_iters, use_backtracking, backtrack_coeff,
                max_backtrack_try, lr0, on_accept)
        else:
            states, actions, real_traj_lengths, next_states, distances, indices = batch
            res = off_policy_optimization(
                optimizer, behavioral_policy, target_policy, last_valid_target_policy, states,
                actions, num_traj, real_traj_lengths, distances, indices, k, G, B, ns, eps,
                kl_threshold, max_off_iters, use_backtracking, backtrack_coeff, max_backtrack_try,
                lr0, on_accept)
        entropy, num_off_iters, backtrack_iter, learning_rate = res
        if torch.isnan(entropy) or torch.isinf(entropy):
            print("Aborting because final entropy is nan or inf...")
            print("There is most likely a problem in knn aliasing. Use a higher k.")
            raise SystemExit(0)
        epoch += 1
        behavioral_policy.load_state_dict(last_valid_target_policy.state_dict())
        target_policy.load_state_dict(last_valid_target_policy.state_dict())
        loss = -_np(entropy)
        entropy = _np(entropy)
        execution_time = time.time() - t0

        heatmap_entropy, heatmap_image = None, None
        if epoch % heatmap_every == 0:
            heatmap_entropy, heatmap_image = heatmap()
            full_entropy = no_grad_entropy(
                collect(num_traj * full_entropy_traj_scale, full_entropy_k),
                num_traj * full_entropy_traj_scale, full_entropy_k, full_B)
            full_entropy = _np(full_entropy)
            if rank == 0:
                _save_policy(behavioral_policy, os.path.join(out_path, f"{epoch}-policy"))
        log_epoch_statistics(writer=writer, log_file=log_file, csv_file_1=csv_file_1,
                             csv_file_2=csv_file_2, epoch=epoch, loss=loss, entropy=entropy,
                             execution_time=execution_time, num_off_iters=num_off_iters,
                             full_entropy=full_entropy, heatmap_image=heatmap_image,
                             heatmap_entropy=heatmap_entropy,
                             backtrack_iters=backtrack_iter, backtrack_lr=learning_rate)
    return behavioral_policy


def off_policy_optimization(optimizer, behavioral_policy, target_policy, last_valid_target_policy,
                            states, actions, num_traj, real_traj_lengths, distances, indices, k, G,
                            B, ns, eps, kl_threshold, max_off_iters, use_backtracking,
                            backtrack_coeff, max_backtrack_try, original_lr, on_accept=None,
                            fns=None):
    """The off-policy loop of one epoch with KL acceptance and backtracking (mepol.py:416-483).

    Returns (final entropy of the last valid target as a 0-d tensor, num_off_iters,
    backtrack_iter, learning_rate).  last_valid_target_policy must hold the behavioral
    parameters on entry (mepol.py:409).  `fns` optionally supplies policy_update / compute_kl /
    compute_entropy with this module's signatures (the sharded multi-rank epoch does).
    """
    import sys

    fns = fns if fns is not None else sys.modules[__name__]
    kl_threshold_reached = False
    num_off_iters = 0
    learning_rate = original_lr
    if use_backtracking:
        for param_group in optimizer.param_groups:
            param_group["lr"] = learning_rate
        backtrack_iter = 1
    else:
        backtrack_iter = None

    deferred = hasattr(fns, "policy_update_deferred") and hasattr(fns, "compute_kl_deferred")
    if fns is sys.modules[__name__]:
        # A caller that replaced policy_update / compute_kl (reference-style patching) gets
        # its functions called, not the deferred built-ins.
        deferred = (fns.policy_update, fns.compute_kl) == _BUILTIN_STEP_FNS
    from . import device_loop

    loop = None
    batch = None
    if deferred and hasattr(fns, "make_device_loop"):
        loop = fns.make_device_loop(optimizer, behavioral_policy, target_policy)
    elif deferred and fns is sys.modules[__name__]:
        batch = P.lookup(states, actions, real_traj_lengths, distances, indices)
        if device_loop.supported(batch, behavioral_policy, target_policy, optimizer):
            loop = device_loop.get(target_policy, optimizer, batch, k, G, B, ns, eps)
            if _same_params(target_policy, behavioral_policy):
                # At an epoch's start the target holds the behavioral parameters (mepol.py:409,
                # 493): one forward into the loop's buffers serves as logp_b and as the first
                # replay's activations.
                loop.load(batch)
                batch.seed_behavioral_logp(behavioral_policy, loop.start_from_behavioral())
            else:
                loop.load(batch, batch.behavioral_logp(behavioral_policy))
                loop.refresh()
    # device loop: the parameters before each replay's step are kept on the device (the last
    # accepted ones), so last_valid is only written when a step is rejected and at the end
    shadow = loop is not None and getattr(loop, "tracks_shadow", False)
    last_accepted = False
    while not kl_threshold_reached:
        if loop is not None:
            # policy_update + compute_kl as one graph replay; two scalars come back.  When an
            # accepted step would be followed by another one, that next replay is launched
            # before this one's scalars are read (the GPU does not wait for the host's
            # decision); a rejection cancels it (optimizer moments and step count restored).
            more = (not (use_backtracking and backtrack_iter > 1)
                    and num_off_iters + 1 != max_off_iters)
            H, KL = loop.step(speculate=more) if shadow else loop.step()
            loss, numeric_error, kl, kl_numeric_error = device_loop.kl_flags(H, KL)
            entropy = -loss
        elif deferred:
            # Queue the update and the KL pass, then read all four control scalars at once.
            loss, loss_flag = fns.policy_update_deferred(
                optimizer, behavioral_policy, target_policy, states, actions, num_traj,
                real_traj_lengths, distances, indices, k, G, B, ns, eps)
            kl, kl_flag = fns.compute_kl_deferred(behavioral_policy, target_policy, states,
                                                  actions, num_traj, real_traj_lengths,
                                                  distances, indices, k, eps)
            vals = torch.stack([loss.detach().reshape(()), kl.reshape(()),
                                loss_flag.reshape(()).to(loss.dtype),
                                kl_flag.reshape(()).to(loss.dtype)]).cpu().numpy()
            entropy, kl = -vals[0], vals[1]
            numeric_error, kl_numeric_error = bool(vals[2]), bool(vals[3])
        else:
            loss, numeric_error = fns.policy_update(optimizer, behavioral_policy, target_policy,
                                                    states, actions, num_traj, real_traj_lengths,
                                                    distances, indices, k, G, B, ns, eps)
            entropy = -_np(loss)
            kl, kl_numeric_error = fns.compute_kl(behavioral_policy, target_policy, states,
                                                  actions, num_traj, real_traj_lengths,
                                                  distances, indices, k, eps)
            kl = _np(kl)

        if not numeric_error and not kl_numeric_error and kl <= kl_threshold:
            if not shadow:
                _copy_policy(last_valid_target_policy, target_policy)
            last_accepted = True
            num_off_iters += 1
            if on_accept is not None:
                on_accept(num_off_iters, entropy, kl, learning_rate)
        else:
            last_accepted = False
            if shadow:
                loop.cancel()
                _copy_params(last_valid_target_policy, loop.step_start_params())
            if use_backtracking:
                if not backtrack_iter == max_backtrack_try:
                    _copy_policy(target_policy, last_valid_target_policy)
                    if loop is not None:
                        loop.refresh()
                    learning_rate = original_lr / (backtrack_coeff ** backtrack_iter)
                    for param_group in optimizer.param_groups:
                        param_group["lr"] = learning_rate
                    backtrack_iter += 1
                    continue
            kl_threshold_reached = True

        if use_backtracking and backtrack_iter > 1:
            kl_threshold_reached = True
        if num_off_iters == max_off_iters:
            kl_threshold_reached = True

    if shadow:
        loop.cancel()  # nothing is in flight here; kept as a guard
        if last_accepted:
            _copy_policy(last_valid_target_policy, target_policy)
            # the last replay's forward ran at exactly these parameters: its logp serves the
            # final entropy's forward of last_valid (mepol.py:466-468)
            seed = batch.seed_behavioral_logp if batch is not None else getattr(
                fns, "seed_behavioral_logp", None)
            if seed is not None:
                seed(last_valid_target_policy, loop.logp_of_last_step())
    with torch.no_grad():
        entropy = fns.compute_entropy(last_valid_target_policy, last_valid_target_policy, states,
                                      actions, num_traj, real_traj_lengths, distances, indices, k,
                                      G, B, ns, eps)
    return entropy, num_off_iters, backtrack_iter, learning_rate


_BUILTIN_STEP_FNS = (policy_update, compute_kl)


def _same_params(a, b):
    """True when two policies hold bitwise equal parameters (one host synchronisation)."""
    pa, pb = list(a.parameters()), list(b.parameters())
    if len(pa) != len(pb) or any(x.shape != y.shape or x.dtype != y.dtype for x, y in zip(pa, pb)):
        return False
    with torch.no_grad():
        fa = torch.cat([x.reshape(-1) for x in pa])
        fb = torch.cat([y.reshape(-1) for y in pb])
        return bool(torch.equal(fa, fb))


def _copy_params(dst, tensors):
    """dst's parameters <- tensors (same order and shapes), one fused device copy."""
    with torch.no_grad():
        torch._foreach_copy_(list(dst.parameters()), list(tensors))


def _copy_policy(dst, src):
    """dst.load_state_dict(src.state_dict()) (mepol.py:443,456) as one fused device copy."""
    dp, sp = list(dst.parameters()), list(src.parameters())
    if len(dp) != len(sp) or list(dst.buffers()) or list(src.buffers()):
        dst.load_state_dict(src.state_dict())
        return
    with torch.no_grad():
        torch._foreach_copy_(dp, sp)


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return x


def _sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()
