"""Calibrate bench.py's CPU baseline (the oracle restatement) against the reference itself.

Runs HERE only (it imports the read-only reference at /root/reference through the shims of
tests/golden/ref_stubs.py; nothing of the reference travels to the GPU box).  For the SURVEY
§8d calibration configs it times, on the same host threads:

  reference   src.algorithms.mepol.collect_particles (per-step batch-1 predict + env.step),
              sklearn NearestNeighbors(k+1).fit(X).kneighbors(X) at full N (mepol.py:190-192),
              policy_update (mepol.py:268-281) and compute_kl (mepol.py:157-174) at full N;
  restatement bench.cpu_baseline(cfg) -- the exact function bench.py runs on the GPU box
              (sampled rollout / k-NN scaled to N, oracle policy_update / compute_kl);

and writes profiles/cpu_calibration.json with per-component and per-epoch ratios
restatement / reference (SURVEY §8d target: 1.0 +- 0.15).  The epoch is
rollout + k-NN + iters x (policy_update + compute_kl) + one final compute_kl-sized pass, with
iters = 30 (max_off_iters of every shipped script).

    python tools/calibrate_cpu_baseline.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
CONFIGS = {
    # C1 MountainCar (scripts/tae/mountain_car.sh): 20 x 400, k = 4, [300, 300], a = 1
    "C1": dict(env="MountainCar", num_traj=20, traj_len=400, nf=2, a=1, hidden=[300, 300], k=4,
               d=2, lr=1e-4, log_std_init=-0.5, max_off_iters=30),
    # C2 GridWorld: 20 x 1000, k = 4, [300, 300], a = 2
    "C2": dict(env="GridWorld", num_traj=20, traj_len=1000, nf=2, a=2, hidden=[300, 300], k=4,
               d=2, lr=1e-5, log_std_init=-1.5, max_off_iters=30),
    # C3 at N = 50k (100 x 500), d = 29, k = 30, [400, 300], a = 8 (no rollout: MuJoCo)
    "C3@50k": dict(num_traj=100, traj_len=500, nf=29, a=8, hidden=[400, 300], k=30, d=29,
                   lr=1e-5, log_std_init=-0.5, max_off_iters=30),
}


def timed(fn, reps=1):
    fn()  # warm (allocator, thread pool)
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t) / reps


def reference_components(cfg, M, envs, GaussianPolicy, torch, threads):
    import scipy.special
    from sklearn.neighbors import NearestNeighbors

    nt, T, nf, a, k, d = (cfg[x] for x in ("num_traj", "traj_len", "nf", "a", "k", "d"))
    N = nt * T
    rng = np.random.default_rng(0)
    torch.manual_seed(0)
    beh = GaussianPolicy(cfg["hidden"], nf, a, log_std_init=cfg["log_std_init"])
    tgt = GaussianPolicy(cfg["hidden"], nf, a, log_std_init=cfg["log_std_init"])
    tgt.load_state_dict(beh.state_dict())
    out = {}
    if cfg.get("env"):
        env = envs[cfg["env"]]()
        env.seed(0)
        nsamp = 4
        out["rollout"] = timed(lambda: M.collect_particles(env, beh, nsamp, T, None)) * nt / nsamp
        lo, hi = ((-1.2, 0.6) if cfg["env"] == "MountainCar" else (-6, 6))
        X = rng.uniform(lo, hi, (N, d)).astype(np.float32)
    else:
        out["rollout"] = 0.0
        X = rng.standard_normal((N, d)).astype(np.float32)

    def knn():
        nbrs = NearestNeighbors(n_neighbors=k + 1, metric="euclidean", algorithm="auto",
                                n_jobs=threads)
        nbrs.fit(X)
        return nbrs.kneighbors(X)

    out["knn"] = timed(knn)
    S = torch.as_tensor(rng.standard_normal((nt, T + 1, nf)), dtype=torch.float64)
    A = torch.as_tensor(0.5 * rng.standard_normal((nt, T, a)), dtype=torch.float64)
    rtl = torch.full((nt, 1), T, dtype=torch.int64)
    I = torch.as_tensor(rng.integers(0, N, (N, k + 1)), dtype=torch.int64)
    D = torch.as_tensor(rng.random((N, k + 1)) + 1.0, dtype=torch.float64)
    B = float(np.log(k) - scipy.special.digamma(k))
    G = float(scipy.special.gamma(d / 2 + 1))
    opt = torch.optim.Adam(tgt.parameters(), lr=cfg["lr"])
    out["policy_update"] = timed(lambda: M.policy_update(opt, beh, tgt, S, A, nt, rtl, D, I, k, G,
                                                         B, d, 0.0), reps=2)
    with torch.no_grad():
        out["compute_kl"] = timed(lambda: M.compute_kl(beh, tgt, S, A, nt, rtl, D, I, k, 0.0),
                                  reps=2)
    return out


def epoch(c, iters):
    return c["rollout"] + c["knn"] + iters * (c["policy_update"] + c["compute_kl"]) + \
        c["compute_kl"]


def main():
    if not os.path.isdir(REF):
        print("reference not present; nothing to do")
        return
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, ROOT)
    import ref_stubs

    ref_stubs.install(REF)
    import torch

    import bench
    import src.algorithms.mepol as M
    from src.envs.gridworld_continuous import GridWorldContinuous
    from src.envs.mountain_car_wall import MountainCarContinuous
    from src.envs.wrappers import ErgodicEnv
    from src.policy import GaussianPolicy

    envs = {"GridWorld": lambda: ErgodicEnv(GridWorldContinuous()),
            "MountainCar": lambda: ErgodicEnv(MountainCarContinuous())}
    threads, aff = bench._cpu_threads()
    torch.set_num_threads(threads)
    result = {"host": bench._cpu_model(), "threads": threads, "configs": {}}
    ratios = []
    for name, cfg in CONFIGS.items():
        iters = cfg["max_off_iters"]
        ref = reference_components(cfg, M, envs, GaussianPolicy, torch, threads)
        port = bench.cpu_baseline(dict(cfg, eps=0.0), 16000, [iters])
        torch.set_num_threads(threads)
        pc = port["components_s"]
        comp = {key: {"reference_s": round(ref[key], 4), "restatement_s": pc[key],
                      "ratio": (round(pc[key] / ref[key], 3) if ref[key] > 0 else None)}
                for key in ("rollout", "knn", "policy_update", "compute_kl")}
        e_ref, e_port = epoch(ref, iters), port["value"]
        ratio = e_port / e_ref
        ratios.append(ratio)
        result["configs"][name] = {"components": comp, "epoch_reference_s": round(e_ref, 3),
                                   "epoch_restatement_s": e_port, "epoch_ratio": round(ratio, 3),
                                   "sample": port["sample"]}
        print(name, json.dumps(result["configs"][name]), flush=True)
    result["epoch_ratio_summary"] = {n: result["configs"][n]["epoch_ratio"] for n in CONFIGS}
    result["target"] = "1.0 +- 0.15 (SURVEY 8d)"
    with open(os.path.join(ROOT, "profiles", "cpu_calibration.json"), "w") as f:
        json.dump(result, f, indent=1)


if __name__ == "__main__":
    main()
