"""Generate the golden fixtures under tests/golden/ by running the REFERENCE implementation.

Test infrastructure only.  Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

It imports the read-only reference (with the shims of ``ref_stubs.py``) and calls the
reference's own functions; it no-ops when /root/reference is absent (e.g. on the GPU box).
Nothing from the reference is copied: only inputs and the outputs the reference produced
are written, as compressed ``.npz`` data files.

Fixtures:
  knn_*.npz        particles -> (D, I) of ``NearestNeighbors(k+1).fit(X).kneighbors(X)``
                   (src/algorithms/mepol.py:190-192) with algorithm='kd_tree', which is what
                   the pinned scikit-learn 0.22 'auto' picks (exact f64 sum of squares).
  entropy_*.npz    compute_importance_weights / compute_entropy / compute_kl / policy_update
                   (mepol.py:114-174, 268-281) over 3 Adam steps: w, H, KL, flags, grads.
  policy_*.npz     GaussianPolicy state dict + get_log_p / forward(deterministic)
                   (src/policy.py:16-67), incl. the pretrained/grid_world weights.
  env_*.npz        MountainCar / GridWorld single steps (mountain_car_wall.py:13-45,
                   gridworld_continuous.py:128-154), edge cases included.
  control_*.npz    mepol() off-policy control flow (mepol.py:404-499) driven by scripted
                   (loss, KL) sequences: learning rates, accepts, backtracks, CSV rows.
  heatmap_*.npz    get_heatmap (mepol.py:19-67) + Discretizer (src/envs/discretizer.py) over
                   scripted visits: average distribution and average discrete entropy.
"""
import io
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path) / 1e3:.0f} kB")


def _knn_ref(X, kp1):
    # Same call as src/algorithms/mepol.py:190-192, pinned-version algorithm choice.
    from sklearn.neighbors import NearestNeighbors

    nbrs = NearestNeighbors(n_neighbors=kp1, metric="euclidean", algorithm="kd_tree", n_jobs=1)
    nbrs.fit(X)
    D, I = nbrs.kneighbors(X)
    return D.astype(np.float64), I.astype(np.int32)


def _sd_arrays(policy, prefix):
    return {f"{prefix}{k}": v.detach().cpu().numpy().copy() for k, v in policy.state_dict().items()}


def gen_knn(M, GridWorldContinuous, ErgodicEnv, GaussianPolicy, train_supervised, torch):
    cases = [
        ("knn_mc_d2", 5000, 2, 5, 0),
        ("knn_d7", 3000, 7, 5, 1),
        ("knn_ant_d29", 2000, 29, 31, 2),
        ("knn_hum_d47", 1500, 47, 31, 3),
        ("knn_hr_d63", 1200, 63, 51, 4),
        ("knn_d30_k30", 1000, 30, 31, 5),
    ]
    for name, n, d, kp1, seed in cases:
        X = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
        D, I = _knn_ref(X, kp1)
        _save(f"{name}.npz", X=X, D=D, I=I, kp1=np.int64(kp1))

    # Real GridWorld particles (exact duplicates present: wall-blocked steps keep the state).
    torch.manual_seed(7)
    np.random.seed(7)
    env = ErgodicEnv(GridWorldContinuous())
    env.init_states.seed(7)
    env.observation_space.seed(7)
    pol = train_supervised(env, GaussianPolicy([300, 300], 2, 2, -1.5), 100, 5000)
    for name, nt, T, kp1 in [("knn_gw_ties", 5, 1000, 5), ("knn_gw_c2", 20, 1000, 5)]:
        _, _, _, ns = M.collect_particles(env, pol, nt, T, None)
        D, I = _knn_ref(ns, kp1)
        _save(f"{name}.npz", X=ns.astype(np.float32), D=D, I=I, kp1=np.int64(kp1))


def gen_entropy(M, GridWorldContinuous, MountainCarContinuous, ErgodicEnv, GaussianPolicy,
                train_supervised, torch, scipy):
    def run_case(name, beh, states, actions, rtl, next_states, k, eps, lr, optimizer="adam"):
        nt = states.shape[0]
        D, I = _knn_ref(next_states.astype(np.float32), k + 1)
        ns = next_states.shape[1]
        B = np.log(k) - scipy.special.digamma(k)
        G = scipy.special.gamma(ns / 2 + 1)
        st = torch.tensor(states, dtype=torch.float64)
        ac = torch.tensor(actions, dtype=torch.float64)
        rl = torch.tensor(rtl, dtype=torch.int64)
        Dt = torch.tensor(D, dtype=torch.float64)
        It = torch.tensor(I, dtype=torch.int64)
        tgt = GaussianPolicy(beh_args["hidden"], beh_args["nf"], beh_args["a"], beh_args["ls"])
        tgt.load_state_dict(beh.state_dict())
        if optimizer == "adam":
            opt = torch.optim.Adam(tgt.parameters(), lr=lr)
        else:
            opt = torch.optim.RMSprop(tgt.parameters(), lr=lr)
        out = dict(states=states, actions=actions, rtl=rtl, next_states=next_states, D=D,
                   I=I, k=np.int64(k), eps=np.float64(eps), ns=np.int64(ns), B=np.float64(B),
                   G=np.float64(G), lr=np.float64(lr), optimizer=np.array(optimizer))
        out.update(_sd_arrays(beh, "beh."))
        for it in range(3):
            out.update(_sd_arrays(tgt, f"it{it}.tgt."))
            with torch.no_grad():
                w = M.compute_importance_weights(beh, tgt, st, ac, nt, rl)
                H = M.compute_entropy(beh, tgt, st, ac, nt, rl, Dt, It, k, G, B, ns, eps)
            out[f"it{it}.w"] = w.numpy().copy()
            out[f"it{it}.H"] = np.float64(H.item())
            loss, nerr = M.policy_update(opt, beh, tgt, st, ac, nt, rl, Dt, It, k, G, B, ns, eps)
            out[f"it{it}.loss"] = np.float64(loss.item())
            out[f"it{it}.nerr"] = np.bool_(bool(nerr))
            for pname, p in tgt.named_parameters():
                out[f"it{it}.grad.{pname}"] = p.grad.detach().numpy().copy()
            with torch.no_grad():
                kl, kerr = M.compute_kl(beh, tgt, st, ac, nt, rl, Dt, It, k, eps)
            out[f"it{it}.kl"] = np.float64(kl.item())
            out[f"it{it}.kerr"] = np.bool_(bool(kerr))
        out.update(_sd_arrays(tgt, "final.tgt."))
        _save(f"{name}.npz", **out)

    # GridWorld rollout, small MLP.
    torch.manual_seed(11)
    np.random.seed(11)
    env = ErgodicEnv(GridWorldContinuous())
    env.init_states.seed(11)
    env.observation_space.seed(11)
    beh_args = dict(hidden=[32, 32], nf=2, a=2, ls=-1.5)
    beh = train_supervised(env, GaussianPolicy(beh_args["hidden"], 2, 2, -1.5), 100, 5000)
    s, a, r, ns = M.collect_particles(env, beh, 4, 200, None)
    run_case("entropy_gw", beh, s, a, r, ns, 12, 0.0, 1e-3)

    # MountainCar rollout (eps = 1e-15 as in experiments/mepol.py:88), RMSprop branch.
    torch.manual_seed(12)
    np.random.seed(12)
    env = ErgodicEnv(MountainCarContinuous())
    env.seed(12)
    beh_args = dict(hidden=[32, 32], nf=2, a=1, ls=-0.5)
    beh = GaussianPolicy(beh_args["hidden"], 2, 1, -0.5)
    s, a, r, ns = M.collect_particles(env, beh, 4, 150, None)
    run_case("entropy_mc", beh, s, a, r, ns, 4, 1e-15, 1e-3, optimizer="rmsprop")

    # Ant-shaped synthetic particles (MuJoCo out of scope): nf=29, a=8, state_filter=range(7).
    torch.manual_seed(13)
    rng = np.random.default_rng(13)
    nt, T, nf, na = 8, 50, 29, 8
    beh_args = dict(hidden=[64, 48], nf=nf, a=na, ls=-0.5)
    beh = GaussianPolicy(beh_args["hidden"], nf, na, -0.5)
    states = rng.standard_normal((nt, T + 1, nf)).astype(np.float32)
    actions = (0.5 * rng.standard_normal((nt, T, na))).astype(np.float32)
    rtl = np.full((nt, 1), T, dtype=np.int32)
    nxt = states[:, 1:, :].reshape(-1, nf)[:, list(range(7))]
    run_case("entropy_ant", beh, states, actions, rtl, nxt, 30, 0.0, 1e-3)

    # Same but the full 29-d state as the k-NN space (BASELINE's d=29).
    torch.manual_seed(14)
    beh = GaussianPolicy(beh_args["hidden"], nf, na, -0.5)
    nxt = states[:, 1:, :].reshape(-1, nf)
    run_case("entropy_ant_d29", beh, states, actions, rtl, nxt, 30, 0.0, 1e-3)

    # GridWorld-size MLP [300,300] (the real architecture).
    torch.manual_seed(15)
    np.random.seed(15)
    env = ErgodicEnv(GridWorldContinuous())
    env.init_states.seed(15)
    env.observation_space.seed(15)
    beh_args = dict(hidden=[300, 300], nf=2, a=2, ls=-1.5)
    beh = train_supervised(env, GaussianPolicy(beh_args["hidden"], 2, 2, -1.5), 100, 5000)
    s, a, r, ns = M.collect_particles(env, beh, 2, 300, None)
    run_case("entropy_gw300", beh, s, a, r, ns, 8, 0.0, 1e-4)

    # Degenerate: exact duplicate particles -> d_k == 0 -> H = -inf, numeric_error (A15/App. A).
    torch.manual_seed(16)
    rng = np.random.default_rng(16)
    beh_args = dict(hidden=[16, 16], nf=2, a=2, ls=-1.5)
    beh = GaussianPolicy(beh_args["hidden"], 2, 2, -1.5)
    nt, T = 2, 40
    states = rng.uniform(-1, 1, (nt, T + 1, 2)).astype(np.float32)
    states[:, 11:31] = states[:, 10:11]  # long blocked stretch: 20 identical states
    actions = (0.1 * rng.standard_normal((nt, T, 2))).astype(np.float32)
    rtl = np.full((nt, 1), T, dtype=np.int32)
    nxt = states[:, 1:, :].reshape(-1, 2)
    run_case("entropy_dup_inf", beh, states, actions, rtl, nxt, 4, 0.0, 1e-3)


def gen_policy(GaussianPolicy, torch):
    torch.manual_seed(21)
    rng = np.random.default_rng(21)
    for name, hidden, nf, na, ls in [("policy_gw", [300, 300], 2, 2, -1.5),
                                     ("policy_ant", [400, 300], 29, 8, -0.5)]:
        p = GaussianPolicy(hidden, nf, na, ls)
        x = rng.standard_normal((64, nf))
        a = rng.standard_normal((64, na))
        with torch.no_grad():
            mean, _ = p(torch.tensor(x), deterministic=True)
            logp = p.get_log_p(torch.tensor(x), torch.tensor(a))
        _save(f"{name}.npz", x=x, a=a, mean=mean.numpy(), logp=logp.numpy(),
              **_sd_arrays(p, "sd."))
    # Pretrained checkpoint shipped with the reference (torch zip, fp32), safe loader only.
    sd = torch.load(os.path.join(REF, "pretrained", "grid_world"), weights_only=True)
    p = GaussianPolicy([300, 300], 2, 2, -1.5)
    p.load_state_dict(sd)
    x = rng.uniform(-6, 6, (64, 2))
    a = 0.2 * rng.standard_normal((64, 2))
    with torch.no_grad():
        mean, _ = p(torch.tensor(x), deterministic=True)
        logp = p.get_log_p(torch.tensor(x), torch.tensor(a))
    _save("policy_pretrained_gw.npz", x=x, a=a, mean=mean.numpy(), logp=logp.numpy(),
          **{f"sd.{k}": v.numpy() for k, v in sd.items()})


def gen_env(GridWorldContinuous, MountainCarContinuous):
    rng = np.random.default_rng(31)
    env = MountainCarContinuous()
    n = 3000
    S = np.stack([rng.uniform(-1.25, 0.65, n), rng.uniform(-0.08, 0.08, n)], 1)
    A = rng.uniform(-2.5, 2.5, (n, 1))
    edge_S = np.array([[-1.2, -0.01], [-1.19, -0.02], [-1.2, 0.01], [0.44, 0.02], [0.45, 0.0],
                       [0.449, 0.001], [0.0, 0.07], [0.0, -0.07], [-0.5, 0.069], [0.6, 0.07]])
    edge_A = np.array([[-1.0], [-5.0], [0.0], [1.0], [1.0], [0.3], [3.0], [-3.0], [1.0], [1.0]])
    S = np.concatenate([edge_S, S])
    A = np.concatenate([edge_A, A])
    NS = np.zeros_like(S)
    for i in range(len(S)):
        env.state = S[i].copy()
        ns, _, _, _ = env.step(A[i])
        NS[i] = ns
    _save("env_mc.npz", S=S, A=A, NS=NS)

    env = GridWorldContinuous()
    n = 6000
    S = rng.uniform(-6, 6, (n, 2)).astype(np.float32)
    A = rng.uniform(-0.4, 0.4, (n, 2))
    edge_S = np.array([[-1.3, 0.0], [5.9, 5.9], [-5.9, -5.9], [0.0, -3.3], [1.24, 2.0],
                       [-2.6, 1.0], [2.6, -1.0], [-3.4, 1.3], [0.0, 3.6], [-1.1, -3.6]],
                      dtype=np.float32)
    edge_A = np.array([[0.2, 0.0], [0.2, 0.2], [-0.2, -0.2], [0.0, 0.2], [0.02, 0.0],
                       [0.2, 0.0], [-0.2, 0.0], [0.0, -0.2], [0.0, -0.2], [0.0, 0.2]])
    S = np.concatenate([edge_S, S])
    A = np.concatenate([edge_A, A])
    NS = np.zeros_like(S)
    for i in range(len(S)):
        env.state = S[i].copy()
        ns, _, _, _ = env.step(A[i])
        NS[i] = ns
    _save("env_gw.npz", S=S, A=A, NS=NS)


def gen_control(M, GaussianPolicy, torch):
    """Drive the reference mepol() loop with scripted (loss, KL) values and record its decisions."""
    scenarios = {
        # kl_threshold = 1.0; each list is the KL returned by successive compute_kl calls.
        "accept_all": dict(kls=[0.1] * 40, nan_loss=[], max_off_iters=5, bt=1),
        "reject_then_bt": dict(kls=[0.1, 0.2, 5.0, 0.3, 0.1, 0.2, 9.0, 9.0, 0.5, 0.1, 0.1, 0.1,
                                    0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1],
                               nan_loss=[], max_off_iters=4, bt=1),
        "first_step_rejected": dict(kls=[7.0, 7.0, 0.2] + [0.1] * 30, nan_loss=[],
                                    max_off_iters=3, bt=1),
        "nan_loss": dict(kls=[0.1, 0.1, 0.1, 0.1] + [0.1] * 30, nan_loss=[1], max_off_iters=3,
                         bt=1),
        "no_backtracking": dict(kls=[0.1, 0.1, 4.0] + [0.1] * 30, nan_loss=[], max_off_iters=6,
                                bt=0),
        "bt_exhausted": dict(kls=[3.0] * 12 + [0.1] * 20, nan_loss=[], max_off_iters=3, bt=1),
    }
    for name, sc in scenarios.items():
        calls = {"update": 0, "kl": 0}
        trace = []

        def fake_collect(env, pol, num_traj, traj_len, state_filter, k, num_workers):
            z = torch.zeros((num_traj, traj_len + 1, 2))
            return (z, z[:, :-1], torch.full((num_traj, 1), traj_len, dtype=torch.int64),
                    None, torch.ones((4, k + 1)), torch.zeros((4, k + 1), dtype=torch.int64))

        def fake_entropy(*a, **kw):
            return torch.tensor(1.25)

        def fake_update(optimizer, beh, tgt, *a, **kw):
            i = calls["update"]
            calls["update"] += 1
            lr = optimizer.param_groups[0]["lr"]
            with torch.no_grad():
                for p in tgt.parameters():
                    p.add_(1.0)  # visible parameter change -> lets us see restores
            loss = torch.tensor(float("nan")) if i in sc["nan_loss"] else torch.tensor(-1.0 - i)
            trace.append(("update", i, lr))
            return loss, bool(torch.isnan(loss))

        def fake_kl(beh, tgt, *a, **kw):
            i = calls["kl"]
            calls["kl"] += 1
            v = sc["kls"][i]
            trace.append(("kl", i, v, float(tgt.log_std.detach()[0])))
            return torch.tensor(v), False

        saved = (M.collect_particles_and_compute_knn, M.compute_entropy, M.policy_update,
                 M.compute_kl)
        M.collect_particles_and_compute_knn = fake_collect
        M.compute_entropy = fake_entropy
        M.policy_update = fake_update
        M.compute_kl = fake_kl
        try:
            class _Env:
                num_features = 2

                def seed(self, s):
                    pass

            def create_policy(is_behavioral=False):
                return GaussianPolicy([4], 2, 2, 0.0)

            with tempfile.TemporaryDirectory() as out:
                buf = io.StringIO()
                old = sys.stdout
                sys.stdout = buf
                try:
                    M.mepol(env=_Env(), env_name="Scripted", state_filter=None,
                            create_policy=create_policy, k=4, kl_threshold=1.0,
                            max_off_iters=sc["max_off_iters"], use_backtracking=sc["bt"],
                            backtrack_coeff=2, max_backtrack_try=4, eps=0.0,
                            learning_rate=0.01, num_traj=2, traj_len=3, num_epochs=2,
                            optimizer="adam", full_entropy_traj_scale=1, full_entropy_k=4,
                            heatmap_every=1000, heatmap_discretizer=None, heatmap_episodes=1,
                            heatmap_num_steps=1, heatmap_cmap=None, heatmap_labels=None,
                            heatmap_interp=None, seed=0, out_path=out, num_workers=1)
                finally:
                    sys.stdout = old
                # execution_time (the last column) is wall clock: zeroed, so a regeneration
                # reproduces every fixture bit-identically (tests compare the other columns)
                csv1 = "".join(
                    line if i == 0 else ",".join(line.rstrip("\n").split(",")[:-1] + ["0"]) + "\n"
                    for i, line in enumerate(open(os.path.join(out, "Scripted.csv"))))
                csv3 = open(os.path.join(out, "Scripted_off_policy_iter.csv")).read()
        finally:
            (M.collect_particles_and_compute_knn, M.compute_entropy, M.policy_update,
             M.compute_kl) = saved
        _save(f"control_{name}.npz", scenario=np.array(json.dumps(sc)),
              trace=np.array(json.dumps(trace)), csv1=np.array(csv1), csv3=np.array(csv3))


def gen_heatmap(M):
    """get_heatmap (mepol.py:19-67) with the reference's Discretizer over scripted visits: a
    replay env hands back fixed states (30 % exactly on bin edges, some outside the ranges)
    and the policy's action is ignored, so the fixture pins binning, averaging and entropy."""
    import matplotlib

    matplotlib.use("Agg")
    import torch
    from src.envs.discretizer import Discretizer

    class Replay:
        def __init__(self, visits):
            self.visits, self.ep, self.t = visits, -1, 0

        def reset(self):
            self.ep += 1
            self.t = 0
            return np.zeros_like(self.visits[0, 0])

        def step(self, a):
            s = self.visits[self.ep, self.t]
            self.t += 1
            return s, 0.0, False, {}

    class Still:
        def predict(self, s, deterministic=False):
            return torch.zeros(1, dtype=torch.float64)

    rng = np.random.default_rng(11)
    E, T = 6, 250
    cases = [("mc", [[-1.2, 0.6], [-0.07, 0.07]], [12, 11], 2, False, np.float64),
             ("gw", [[-6.0, 6.0], [-6.0, 6.0]], [20, 20], 2, False, np.float32),
             ("xy", [[-12.0, 12.0], [-12.0, 12.0]], [40, 40], 5, True, np.float64)]
    for name, ranges, bins, nf, xy, dt in cases:
        cols = []
        for (lo, hi), nb in zip(ranges, bins):
            edges = np.linspace(lo, hi, nb + 1)
            x = rng.uniform(lo - 0.1 * (hi - lo), hi + 0.1 * (hi - lo), E * T)
            pick = rng.random(E * T) < 0.3
            x[pick] = rng.choice(edges, int(pick.sum()))
            cols.append(x)
        vis = np.stack(cols, 1)
        if nf > 2:
            vis = np.concatenate([vis, rng.standard_normal((E * T, nf - 2))], 1)
        vis = vis.astype(dt).reshape(E, T, nf)
        disc = Discretizer(ranges, bins, (lambda s: [s[0], s[1]]) if xy else None)
        dist, ent, _ = M.get_heatmap(Replay(vis), Still(), disc, E, T, "Blues", None, ("X", "Y"))
        _save(f"heatmap_{name}.npz", visits=vis, ranges=np.array(ranges, np.float64),
              bins=np.array(bins), xy=np.array(xy), dist=np.asarray(dist, np.float64),
              entropy=np.array(float(ent)))


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return
    only = set(sys.argv[1:])  # e.g. `make_golden.py heatmap` regenerates one family
    sys.path.insert(0, HERE)
    import ref_stubs

    ref_stubs.install(REF)
    import scipy.special
    import torch

    import src.algorithms.mepol as M
    from src.envs.gridworld_continuous import GridWorldContinuous
    from src.envs.mountain_car_wall import MountainCarContinuous
    from src.envs.wrappers import ErgodicEnv
    from src.policy import GaussianPolicy, train_supervised

    torch.set_num_threads(8)
    if not only or "env" in only:
        gen_env(GridWorldContinuous, MountainCarContinuous)
    if not only or "policy" in only:
        gen_policy(GaussianPolicy, torch)
    if not only or "knn" in only:
        gen_knn(M, GridWorldContinuous, ErgodicEnv, GaussianPolicy, train_supervised, torch)
    if not only or "entropy" in only:
        gen_entropy(M, GridWorldContinuous, MountainCarContinuous, ErgodicEnv, GaussianPolicy,
                    train_supervised, torch, scipy)
    if not only or "control" in only:
        gen_control(M, GaussianPolicy, torch)
    if not only or "heatmap" in only:
        gen_heatmap(M)


if __name__ == "__main__":
    main()
