"""CPU restatement of the reference MEPOL hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it, only as the checker / CPU baseline.  The product (mepol_amd/) never
imports it and has no CPU fallback.

It restates the reference algorithm (RiccZamboni/mepol, src/algorithms/mepol.py) in float64
numpy / torch-CPU, deliberately in the reference's own shape (per-trajectory loops, behavioral
log-probs recomputed every call) so that it also serves as the CPU wall-clock baseline.
Pinned against the golden fixtures in tests/golden/ produced by running the reference itself
(tests/golden/make_golden.py); see tests/test_oracle_golden.py.
"""
import ctypes
import math
import os
import subprocess

import numpy as np
import torch


# -------------------------------------------------------------------------------------------
# k-NN  (src/algorithms/mepol.py:190-192; sklearn kd_tree arithmetic)
# -------------------------------------------------------------------------------------------
def knn_exact(X, kp1, Q=None, chunk=512):
    """Exact k-NN by brute force: d^2 = sum_f (q_f - x_f)^2 in f64 (feature order), rows sorted by
    (distance, index).  Returns (D f64 [nq, kp1], I int64 [nq, kp1])."""
    X = np.asarray(X, dtype=np.float32).astype(np.float64)
    Q = X if Q is None else np.asarray(Q, dtype=np.float32).astype(np.float64)
    n, d = X.shape
    nq = Q.shape[0]
    D = np.empty((nq, kp1), dtype=np.float64)
    I = np.empty((nq, kp1), dtype=np.int64)
    idx = np.arange(n)
    for s in range(0, nq, chunk):
        q = Q[s:s + chunk]
        acc = np.zeros((q.shape[0], n), dtype=np.float64)
        for f in range(d):
            t = q[:, f:f + 1] - X[None, :, f]
            acc += t * t
        part = np.argpartition(acc, kp1 - 1, axis=1)[:, :kp1] if kp1 < n else np.tile(idx, (q.shape[0], 1))
        # exact boundary handling: include every candidate tied with the kp1-th value
        for r in range(q.shape[0]):
            row = acc[r]
            kth = row[part[r]].max()
            cand = np.nonzero(row <= kth)[0]
            order = np.lexsort((cand, row[cand]))[:kp1]
            sel = cand[order]
            D[s + r] = np.sqrt(row[sel])
            I[s + r] = sel
    return D, I


def knn_exact_sampled(X, kp1, Q, chunk=64):
    """knn_exact for a few queries Q against a large candidate set X (N up to 500k).

    Same result as knn_exact (feature-order f64 distances, (distance, index) order); the
    candidates are pre-screened with the f64 GEMM form |q|^2 + |x|^2 - 2 q.x, whose error is
    below (d + 4) * 2^-52 * (|q| + |x|)^2 <= tol (Higham's dot-product bound with margin), so
    every candidate whose exact d^2 is at most the kp1-th exact value survives the screen:
    approx(c) <= exact(c) + tol <= exact_kp1 + tol <= approx_kp1 + 2 tol."""
    X = np.asarray(X, dtype=np.float32).astype(np.float64)
    Q = np.asarray(Q, dtype=np.float32).astype(np.float64)
    n, d = X.shape
    xn = np.einsum("ij,ij->i", X, X)
    qn = np.einsum("ij,ij->i", Q, Q)
    scale = (np.sqrt(qn).max() + np.sqrt(xn).max()) ** 2
    tol = (d + 4) * 2.0 ** -52 * scale * 4
    D = np.empty((Q.shape[0], kp1), dtype=np.float64)
    I = np.empty((Q.shape[0], kp1), dtype=np.int64)
    for s in range(0, Q.shape[0], chunk):
        q = Q[s:s + chunk]
        approx = qn[s:s + chunk, None] + xn[None, :] - 2.0 * (q @ X.T)
        kth = np.partition(approx, kp1 - 1, axis=1)[:, kp1 - 1]
        for r in range(q.shape[0]):
            cand = np.nonzero(approx[r] <= kth[r] + 2 * tol)[0]
            acc = np.zeros(cand.shape[0])
            for f in range(d):
                t = q[r, f] - X[cand, f]
                acc += t * t
            order = np.lexsort((cand, acc))[:kp1]
            D[s + r] = np.sqrt(acc[order])
            I[s + r] = cand[order]
    return D, I


def knn_sklearn(X, kp1, n_jobs=1, algorithm="auto"):
    """The reference call itself (mepol.py:190-192) -- used as the timed CPU baseline."""
    from sklearn.neighbors import NearestNeighbors

    nbrs = NearestNeighbors(n_neighbors=kp1, metric="euclidean", algorithm=algorithm, n_jobs=n_jobs)
    nbrs.fit(X)
    return nbrs.kneighbors(X)


# -------------------------------------------------------------------------------------------
# Policy  (src/policy.py:43-61)
# -------------------------------------------------------------------------------------------
def mlp_mean(sd, x):
    """mean = W_m relu(... relu(W_0 x + b_0) ...) + b_m from a GaussianPolicy state dict."""
    h = np.asarray(x, dtype=np.float64)
    i = 0
    while f"net.{i}.weight" in sd:
        h = np.maximum(h @ np.asarray(sd[f"net.{i}.weight"], np.float64).T
                       + np.asarray(sd[f"net.{i}.bias"], np.float64), 0.0)
        i += 2
    return h @ np.asarray(sd["mean.weight"], np.float64).T + np.asarray(sd["mean.bias"], np.float64)


def log_p(sd, states, actions):
    """policy.py:43-51 with eps = 1e-7 (dtypes.py:7)."""
    mu = mlp_mean(sd, states)
    ls = np.asarray(sd["log_std"], np.float64)
    return np.sum(-0.5 * (np.log(2 * np.pi) + 2 * ls + (np.asarray(actions) - mu) ** 2
                          / (np.exp(ls) + 1e-7) ** 2), axis=1)


# -------------------------------------------------------------------------------------------
# IW / entropy / KL / closed-form gradient  (mepol.py:114-174)
# -------------------------------------------------------------------------------------------
def importance_weights(logp_t, logp_b, lengths):
    """Per trajectory exp(cumsum(logp_t - logp_b)) over its real length, concatenated, then
    normalised (mepol.py:119-139).  logp_*: [nt, T]."""
    parts = []
    for n, L in enumerate(lengths):
        parts.append(np.exp(np.cumsum(logp_t[n, :L] - logp_b[n, :L])))
    u = np.concatenate(parts)
    return u / np.sum(u)


def entropy(w, D, I, k, G, B, ns, eps):
    """mepol.py:146-152: uses I[:, :-1] (self + k-1 neighbours) and D[:, k]."""
    W = np.sum(w[I[:, :-1]], axis=1) if I.shape[1] == k + 1 else np.sum(w[I[:, :k]], axis=1)
    V = (D[:, k] ** ns * np.pi ** (ns / 2)) / G
    with np.errstate(divide="ignore", invalid="ignore"):
        return -np.sum((W / k) * np.log(W / (V + eps) + eps)) + B


def kl(w, I, k, eps):
    """mepol.py:161-172 (unclamped value and its numeric-error flag, then the clamp)."""
    W = np.sum(w[I[:, :k]], axis=1)
    N = w.shape[0]
    with np.errstate(divide="ignore", invalid="ignore"):
        v = (1 / N) * np.sum(np.log(k / (N * W) + eps))
    err = bool(np.isinf(v) or np.isnan(v))
    return max(0.0, v), err, v


def entropy_grad_logp(w, D, I, k, G, ns, eps, lengths):
    """dH/dlogp_t[n, s] in closed form, verified against the reference's
    autograd.  Returns a [nt, T] array (zeros past each real length)."""
    N = w.shape[0]
    W = np.sum(w[I[:, :k]], axis=1)
    V = (D[:, k] ** ns * np.pi ** (ns / 2)) / G
    r = W / (V + eps)
    with np.errstate(divide="ignore", invalid="ignore"):
        g = -(1.0 / k) * (np.log(r + eps) + r / (r + eps))
    gamma = np.zeros(N)
    np.add.at(gamma, I[:, :k].reshape(-1), np.repeat(g, k))
    S = np.dot(gamma, w)
    c = (gamma - S) * w
    T = max(lengths)
    out = np.zeros((len(lengths), T))
    p = 0
    for n, L in enumerate(lengths):
        seg = c[p:p + L]
        out[n, :L] = np.cumsum(seg[::-1])[::-1]
        p += L
    return out


# -------------------------------------------------------------------------------------------
# Environments  (mountain_car_wall.py:13-45, gridworld_continuous.py:128-154)
# -------------------------------------------------------------------------------------------
def mountaincar_step(S, A):
    """Vectorised MountainCar step; S f64 [n,2], A [n, >=1]."""
    p = S[:, 0].astype(np.float64).copy()
    v = S[:, 1].astype(np.float64).copy()
    force = np.minimum(np.maximum(A[:, 0].astype(np.float64), -1.0), 1.0)
    v = v + (force * 0.0015 - 0.0025 * np.cos(3 * p))
    v = np.minimum(np.maximum(v, -0.07), 0.07)
    p = p + v
    p = np.minimum(np.maximum(p, -1.2), 0.6)
    v = np.where((p == -1.2) & (v < 0), 0.0, v)
    over = p > 0.45
    p = np.where(over, 0.45, p)
    v = np.where(over, 0.0, v)
    return np.stack([p, v], 1)


GRID_WALLS = [(-1.25, 1.25, -2.5, 2.5), (-2.5, -1.25, -1.25, 1.25), (1.25, 2.5, -1.25, 1.25),
              (-6.0, -3.5, -1.25, 1.25), (-1.25, 1.25, -6.0, -3.5), (3.5, 6.0, -1.25, 1.25),
              (-1.25, 1.25, 3.5, 6.0)]


def gridworld_step(S, A):
    """Vectorised GridWorld step; S f32 [n,2], A f64 [n,2] -> f32 [n,2]."""
    x = S[:, 0].astype(np.float64)
    y = S[:, 1].astype(np.float64)
    nx = x + np.clip(A[:, 0].astype(np.float64), -0.2, 0.2)
    ny = y + np.clip(A[:, 1].astype(np.float64), -0.2, 0.2)
    hit = np.zeros(len(S), dtype=bool)
    for (x0, x1, y0, y1) in GRID_WALLS:
        hit |= (x0 <= nx) & (nx <= x1) & (y0 <= ny) & (ny <= y1)
    hit |= (np.abs(nx) >= 6) | (np.abs(ny) >= 6)
    nx = np.where(hit, x, nx)
    ny = np.where(hit, y, ny)
    return np.stack([nx, ny], 1).astype(np.float32)


def rollout(env, sd, log_std, init, noise, T):
    """Deterministic restatement of collect_particles (mepol.py:76-109) with injected noise.

    env: "mountaincar" | "gridworld"; init [nt, 2]; noise [T, nt, a].
    Returns states f32 [nt, T+1, 2], actions f32 [nt, T, a]."""
    nt = init.shape[0]
    a_dim = noise.shape[2]
    states = np.zeros((nt, T + 1, 2), np.float32)
    actions = np.zeros((nt, T, a_dim), np.float32)
    s = init.astype(np.float64) if env == "mountaincar" else init.astype(np.float32)
    states[:, 0] = s
    std = np.exp(np.asarray(log_std, np.float64))
    for t in range(T):
        a = mlp_mean(sd, s.astype(np.float64)) + noise[t] * std
        actions[:, t] = a
        s = mountaincar_step(s, a) if env == "mountaincar" else gridworld_step(s, a)
        states[:, t + 1] = s
    return states, actions


_NATIVE = {}


def _native():
    """oracle/native/librollout_kordered.so (gcc; `make` builds it, else built here)."""
    if "lib" not in _NATIVE:
        here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")
        src = os.path.join(here, "rollout_kordered.c")
        so = os.path.join(here, "librollout_kordered.so")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared", src, "-o", so,
                            "-lm"], check=True)
        lib = ctypes.CDLL(so)
        vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
        lib.rollout_kordered.argtypes = [ci, i64, i64, ci, ci, ci, ci] + [vp] * 12
        lib.rollout_kordered.restype = ci
        _NATIVE["lib"] = lib
    return _NATIVE["lib"]


def rollout_kordered(env, sd, std, init, noise, T, k_chunks=1):
    """collect_particles (mepol.py:76-109) for the 2 -> [h0, h1] -> a ReLU policy with the MLP
    summed in the documented k-ordered / butterfly order of oracle/native/rollout_kordered.c
    (the order the HIP rollout kernels commit to), so actions compare bit for bit; k_chunks =
    the k-ranges of the second layer's sum (ops.rollout_mlp_plan reports the kernel's).
    std: exp(log_std) [a] f64; init [nt, 2] (f64 MountainCar, f32 GridWorld); noise [T, nt, a].
    Returns states f32 [nt, T+1, 2], actions f32 [nt, T, a]."""
    def arr(x, dt):
        return np.ascontiguousarray(np.asarray(x, dtype=dt))

    W1, b1 = arr(sd["net.0.weight"], np.float64), arr(sd["net.0.bias"], np.float64)
    W2, b2 = arr(sd["net.2.weight"], np.float64), arr(sd["net.2.bias"], np.float64)
    Wm, bm = arr(sd["mean.weight"], np.float64), arr(sd["mean.bias"], np.float64)
    h0, h1, a_dim = W1.shape[0], W2.shape[0], Wm.shape[0]
    nt = init.shape[0]
    mc = env == "mountaincar"
    i64 = arr(init, np.float64) if mc else None
    i32 = None if mc else arr(init, np.float32)
    nz = arr(noise, np.float64)
    sdv = arr(std, np.float64)
    states = np.zeros((nt, T + 1, 2), np.float32)
    actions = np.zeros((nt, T, a_dim), np.float32)
    p = lambda x: None if x is None else x.ctypes.data  # noqa: E731
    rc = _native().rollout_kordered(0 if mc else 1, nt, T, h0, h1, a_dim, int(k_chunks), p(W1),
                                    p(b1), p(W2),
                                    p(b2), p(Wm), p(bm), p(sdv), p(i64), p(i32), p(nz),
                                    p(states), p(actions))
    assert rc == 0
    return states, actions


# -------------------------------------------------------------------------------------------
# Visitation heatmap  (src/algorithms/mepol.py:26-47, src/envs/discretizer.py:4-26)
# -------------------------------------------------------------------------------------------
def heatmap_stats(ranges, bins_sizes, visits):
    """get_heatmap's statistics over recorded visits [E, T, nf] (nf = len(bins_sizes), already
    the discretized features): per-episode np.digitize bin counts / T, their average, and the
    average scipy.stats.entropy, accumulated episode by episode as the reference does."""
    import scipy.stats

    edges = [np.linspace(ranges[i][0], ranges[i][1], bins_sizes[i] + 1)[1:-1]
             for i in range(len(bins_sizes))]
    E, T = visits.shape[0], visits.shape[1]
    avg = np.zeros(bins_sizes)
    avg_h = 0.0
    for e in range(E):
        dist = np.zeros(bins_sizes)
        for t in range(T):
            s = visits[e, t]
            dist[tuple(np.digitize(x=s[i], bins=edges[i]) for i in range(len(s)))] += 1
        dist /= T
        avg += dist
        avg_h += scipy.stats.entropy(dist.ravel())
    return avg / E, avg_h / E


# -------------------------------------------------------------------------------------------
# Timed CPU baseline: one MEPOL off-policy iteration in the reference's own shape
# -------------------------------------------------------------------------------------------
class TorchPolicy(torch.nn.Module):
    """CPU float64 Gaussian MLP with the reference's forward (policy.py:43-61)."""

    def __init__(self, hidden, nf, a, log_std_init=-0.5):
        super().__init__()
        layers = []
        w = [nf] + list(hidden)
        for i, o in zip(w[:-1], w[1:]):
            layers += [torch.nn.Linear(i, o, dtype=torch.float64), torch.nn.ReLU()]
        self.net = torch.nn.Sequential(*layers)
        self.mean = torch.nn.Linear(w[-1], a, dtype=torch.float64)
        self.log_std = torch.nn.Parameter(torch.full((a,), log_std_init, dtype=torch.float64))

    def forward(self, x, deterministic=False):
        """(mean, sample) as policy.py:53-61: the sample is drawn even when only the mean is
        used (get_log_p), which is part of the reference's cost."""
        mu = self.mean(self.net(x))
        if deterministic:
            return mu, mu
        return mu, mu + torch.randn(mu.size(), dtype=torch.float64) * torch.exp(self.log_std)

    def predict(self, s, deterministic=False):
        """policy.py:64-67: batch-1 action for one state."""
        with torch.no_grad():
            x = torch.tensor(s, dtype=torch.float64).unsqueeze(0)
            return self(x, deterministic=deterministic)[1][0]

    def get_log_p(self, s, a):
        mu, _ = self(s)
        return torch.sum(-0.5 * (math.log(2 * math.pi) + 2 * self.log_std
                                 + (a - mu) ** 2 / (torch.exp(self.log_std) + 1e-7) ** 2), dim=1)


# Scalar (one env, one step) restatements of the env dynamics, in the reference's per-step shape:
# the CPU baseline's rollout times these, as the reference steps one gym env per call.
def gridworld_step_scalar(state, action, dim=6.0, max_delta=0.2):
    """gridworld_continuous.py:128-154 for one env: f32 state [2], f64 action [2]."""
    x, y = state
    nx = x + np.clip(action[0], -max_delta, max_delta)
    ny = y + np.clip(action[1], -max_delta, max_delta)
    for (x0, x1, y0, y1) in GRID_WALLS:
        if x0 <= nx <= x1 and y0 <= ny <= y1:
            nx, ny = x, y
    if np.abs(nx) >= dim or np.abs(ny) >= dim:
        nx, ny = x, y
    return np.array([nx, ny], dtype=np.float32)


def mountaincar_step_scalar(state, action):
    """mountain_car_wall.py:13-45 for one env: f64 state [2]."""
    p, v = float(state[0]), float(state[1])
    v += min(max(action[0], -1.0), 1.0) * 0.0015 - 0.0025 * math.cos(3 * p)
    v = min(max(v, -0.07), 0.07)
    p = min(max(p + v, -1.2), 0.6)
    if p == -1.2 and v < 0:
        v = 0.0
    if p > 0.45:
        p, v = 0.45, 0.0
    return np.array([p, v])


def collect_particles_scalar(step, reset, policy, num_traj, traj_len, nf, a_dim):
    """collect_particles (mepol.py:70-111) in the reference's shape: for every trajectory and
    step one batch-1 policy.predict and one scalar env step, recorded into f32 arrays, then the
    next-state concatenation."""
    states = np.zeros((num_traj, traj_len + 1, nf), dtype=np.float32)
    actions = np.zeros((num_traj, traj_len, a_dim), dtype=np.float32)
    for n in range(num_traj):
        s = reset()
        for t in range(traj_len):
            states[n, t] = s
            a = policy.predict(s).numpy()
            actions[n, t] = a
            s = step(s, a)
        states[n, traj_len] = s
    next_states = np.concatenate([states[n, 1:] for n in range(num_traj)], axis=0)
    return states, actions, next_states


def torch_iw(beh, tgt, states, actions, nt, lengths):
    """compute_importance_weights in the reference's shape (per-trajectory loop, mepol.py:121-138)."""
    out = None
    for n in range(nt):
        L = int(lengths[n])
        lt = tgt.get_log_p(states[n, :L], actions[n, :L])
        lb = beh.get_log_p(states[n, :L], actions[n, :L])
        u = torch.exp(torch.cumsum(lt - lb, dim=0))
        out = u if out is None else torch.cat([out, u], 0)
    return out / torch.sum(out)


def torch_entropy(beh, tgt, states, actions, nt, lengths, D, I, k, G, B, ns, eps):
    w = torch_iw(beh, tgt, states, actions, nt, lengths)
    W = torch.sum(w[I[:, :-1]], dim=1)
    V = (torch.pow(D[:, k], ns) * torch.pow(torch.tensor(np.pi, dtype=torch.float64), ns / 2)) / G
    return -torch.sum((W / k) * torch.log((W / (V + eps)) + eps)) + B


def torch_kl(beh, tgt, states, actions, nt, lengths, I, k, eps):
    w = torch_iw(beh, tgt, states, actions, nt, lengths)
    W = torch.sum(w[I[:, :-1]], dim=1)
    N = w.shape[0]
    v = (1 / N) * torch.sum(torch.log(k / (N * W) + eps))
    return torch.clamp_min(v, 0.0), bool(torch.isinf(v) or torch.isnan(v))


def torch_policy_update(opt, beh, tgt, states, actions, nt, lengths, D, I, k, G, B, ns, eps):
    opt.zero_grad()
    loss = -torch_entropy(beh, tgt, states, actions, nt, lengths, D, I, k, G, B, ns, eps)
    err = bool(torch.isinf(loss) or torch.isnan(loss))
    loss.backward()
    opt.step()
    return loss, err
