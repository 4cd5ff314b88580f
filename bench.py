"""MEPOL epoch benchmark on MI355X (BASELINE.json metric: epoch wall-clock + k-NN GB/s).

Workload (BASELINE configs[2], "C3"): Ant-shaped particle batch, N = 400 trajectories x 500
steps = 200,000 particles, k-NN space d = 29 (full state), k = 30, policy 29 -> [400, 300] -> 8
(f64, as the reference), Adam lr 1e-5, KL threshold 15, 30 off-policy iterations.  MuJoCo is
out of scope, so the rollout phase is replaced by a seeded synthetic batch resident in HBM
(states ~ N(0,1) f32, actions ~ N(0, 0.5^2) f32) -- the same on the CPU baseline leg.

One "step" = one MEPOL epoch inside the reference's timed window (mepol.py:405 -> 499) minus
the rollout: exact k-NN over the next states + the off-policy loop (policy_update +
compute_kl until the stop rule) + the final entropy.

    python bench.py [--gpus N] [--steps K] [--warmup W]
Multi-GPU (one process per GPU, launched by torch.distributed.run): each rank owns
N/world trajectories; next-states are all-gathered over RCCL before the k-NN, each rank answers
its own queries, and the per-iteration scalars / weight vectors / parameter gradients are
reduced so every rank takes the same steps (strong scaling: fixed N = 200k).
"""
import argparse
import json
import os
import platform
import time

import numpy as np
import torch

CFG = dict(num_traj=400, traj_len=500, nf=29, a=8, hidden=[400, 300], k=30, d=29, lr=1e-5,
           kl_threshold=15.0, max_off_iters=30, backtrack_coeff=2, max_backtrack_try=10, eps=0.0)
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector == FP32 matrix peak
PEAK_F16_TFLOPS = 2500.0   # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense
PEAK_HBM_GBPS = 8000.0


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-queries", type=int, default=16000)
    return p.parse_args()


def synthetic_batch(seed, device, rank=0, world=1):
    g = torch.Generator(device=device).manual_seed(seed)
    nt, T, nf, a = CFG["num_traj"], CFG["traj_len"], CFG["nf"], CFG["a"]
    states = torch.randn((nt, T + 1, nf), generator=g, device=device, dtype=torch.float32)
    actions = 0.5 * torch.randn((nt, T, a), generator=g, device=device, dtype=torch.float32)
    per = nt // world
    return states[rank * per:(rank + 1) * per].contiguous(), actions[rank * per:(rank + 1) * per].contiguous()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    # MEPOL_BENCH_SHARDED=1 runs the multi-rank code path (ShardedEpoch + captured RCCL
    # collectives) at world size 1: a one-GPU rehearsal of what --gpus N runs per rank.
    sharded = world > 1 or os.environ.get("MEPOL_BENCH_SHARDED") == "1"
    if sharded:
        import torch.distributed as dist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))

        backend = os.environ.get("MEPOL_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal of the multi-rank path with several ranks on one GPU
            dist.init_process_group(backend)
    import scipy.special

    from mepol_amd import ops
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.policy import GaussianPolicy

    k, nf, a, d = CFG["k"], CFG["nf"], CFG["a"], CFG["d"]
    ns = d
    B = float(np.log(k) - scipy.special.digamma(k))
    G = float(scipy.special.gamma(ns / 2 + 1))
    torch.manual_seed(0)
    behavioral = GaussianPolicy(CFG["hidden"], nf, a, -0.5).to(dev)
    target = GaussianPolicy(CFG["hidden"], nf, a, -0.5).to(dev)
    last_valid = GaussianPolicy(CFG["hidden"], nf, a, -0.5).to(dev)
    target.load_state_dict(behavioral.state_dict())
    last_valid.load_state_dict(behavioral.state_dict())
    opt = torch.optim.Adam(target.parameters(), lr=CFG["lr"])
    N = CFG["num_traj"] * CFG["traj_len"]

    batches = [synthetic_batch(s, dev, rank, world) for s in range(3)]
    knn_events = []
    iters_done = []

    def one_epoch(i):
        states32, actions32 = batches[i % len(batches)]
        nt_local = states32.shape[0]
        T = CFG["traj_len"]
        st = states32.double()
        ac = actions32.double()
        rtl = torch.full((nt_local, 1), T, dtype=torch.int64, device=dev)
        nxt = states32[:, 1:].reshape(-1, nf)[:, :d].contiguous()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        last_valid.load_state_dict(behavioral.state_dict())
        if not sharded:
            e0.record()
            st_, ac_, rl_, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, k)
            e1.record()
            res = M.off_policy_optimization(
                opt, behavioral, target, last_valid, st_, ac_, nt_local, rl_, D, I, k, G, B, ns,
                CFG["eps"], CFG["kl_threshold"], CFG["max_off_iters"], True,
                CFG["backtrack_coeff"], CFG["max_backtrack_try"], CFG["lr"])
        else:
            from mepol_amd.parallel import ShardedEpoch

            ep = ShardedEpoch(st, ac, rtl, nxt, k, dist)
            e0.record()
            ep.build_knn()
            e1.record()
            res = ep.off_policy_optimization(
                opt, behavioral, target, last_valid, G, B, ns, CFG["eps"], CFG["kl_threshold"],
                CFG["max_off_iters"], True, CFG["backtrack_coeff"], CFG["max_backtrack_try"],
                CFG["lr"])
        entropy, n_off, _, _ = res
        behavioral.load_state_dict(last_valid.state_dict())
        target.load_state_dict(last_valid.state_dict())
        _ = float(entropy)
        knn_events.append((e0, e1))
        iters_done.append(n_off)

    for i in range(args.warmup):
        one_epoch(i)
    knn_events.clear()
    iters_done.clear()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one_epoch(args.warmup + i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    epoch_s = elapsed / args.steps
    knn_ms = float(np.mean([a.elapsed_time(b) for a, b in knn_events]))

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    from mepol_amd import parallel
    from mepol_amd.algorithms import device_loop

    it = (parallel._SHARDED_CACHE if sharded else device_loop._CACHE).get(target)
    iteration_path = "hip-graph replay" if it is not None and it.graph is not None else "eager"
    nq = N // world
    F = 3.0 * d * nq * N                      # algorithmic flops
    B_scan = 4.0 * d * nq * N                 # algorithmic scan bytes
    knn_tflops = F / (knn_ms * 1e-3) / 1e12
    # Which selection the library ran (include/mepol_amd.h; MEPOL_KNN_PRECISION=f32 forces f32):
    # split-f16 issues 3 products x 2 x K flops per (query, candidate), K = 16*ceil((d+1)/16).
    if os.environ.get("MEPOL_KNN_PRECISION", "") != "f32" and d + 1 <= 48 and k + 1 <= 60:
        K16 = 16 * ((d + 1 + 15) // 16)
        knn_issued = 3 * 2 * K16 * float(nq) * N
        knn_peak = PEAK_F16_TFLOPS
        knn_desc = "split-f16 MFMA selection (3 products, f32 accumulate) + f64 exact refine (bit-exact output)"
    else:
        knn_issued = 2 * 2 * ((d + 2) // 2) * float(nq) * N
        knn_peak = PEAK_FP32_TFLOPS
        knn_desc = "fp32 MFMA selection + f64 exact refine (bit-exact output)"
    knn_gbps = B_scan / (knn_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "knn_pmc.json")
    if os.path.exists(pmc_path) and world == 1:  # counters were taken on the 1-GPU k-NN call
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    line = {
        "metric": "MEPOL epoch wall-clock (C3 Ant-shaped, N=200k, d=29, k=30; rollout excluded)",
        "value": round(epoch_s, 6),
        "unit": "s/epoch",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(epoch_s * 1e3, 3),
        "higher_is_better": False,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "C3 Ant-shaped MEPOL epoch (k-NN + off-policy loop + final H)",
                   "particles": N, "num_traj": CFG["num_traj"], "traj_len": CFG["traj_len"],
                   "d": d, "k": k, "policy": f"{nf}->{CFG['hidden']}->{a} f64",
                   "off_policy_iters": float(np.mean(iters_done)), "parallelism": f"dp{world}",
                   "knn_precision": knn_desc,
                   "off_policy_iteration": iteration_path},
        "particles_per_s": round(N / epoch_s, 1),
        "knn_ms": round(knn_ms, 3),
        "knn_scan_GBps": round(knn_gbps, 1),
        "knn_scan_frac_of_8TBps": round(knn_gbps / PEAK_HBM_GBPS, 3),
        "roofline": {"bound": "mfma", "achieved": round(knn_tflops, 2), "peak": knn_peak,
                     "unit": "TFLOP/s", "frac": round(knn_tflops / knn_peak, 4),
                     "mfma_issued_tflops": round(knn_issued / (knn_ms * 1e-3) / 1e12, 2),
                     "traffic": traffic,
                     "kernel": "k-NN (norms+pack+select+refine+exact), achieved = F/t with F = 3*d*Nq*Nc (SURVEY 8d); the select is VALU-issue-bound (threshold/merge work), not MFMA-bound"},
    }
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.cpu_sample_queries)
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(sample_queries):
    """The oracle (reference-shaped CPU restatement, torch f64 + sklearn) on host cores.

    Bounded sample: sklearn k-NN for `sample_queries` queries against all 200k candidates
    (scaled by 200k / sample_queries), one policy_update + one compute_kl at full N
    (scaled by the GPU run's iteration count), plus one final-entropy forward."""
    import sklearn
    from sklearn.neighbors import NearestNeighbors

    from oracle import mepol_oracle as O

    cores = min(16, len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    k, nf, a, d = CFG["k"], CFG["nf"], CFG["a"], CFG["d"]
    nt, T = CFG["num_traj"], CFG["traj_len"]
    rng = np.random.default_rng(0)
    X = rng.standard_normal((nt * T, d)).astype(np.float32)
    t = time.perf_counter()
    nbrs = NearestNeighbors(n_neighbors=k + 1, metric="euclidean", algorithm="auto", n_jobs=cores)
    nbrs.fit(X)
    Dq, Iq = nbrs.kneighbors(X[:sample_queries])
    knn_s = (time.perf_counter() - t) * (X.shape[0] / sample_queries)
    # full-N iteration on reference-shaped torch CPU code (per-trajectory loops)
    torch.manual_seed(0)
    beh = O.TorchPolicy(CFG["hidden"], nf, a)
    tgt = O.TorchPolicy(CFG["hidden"], nf, a)
    tgt.load_state_dict(beh.state_dict())
    opt = torch.optim.Adam(tgt.parameters(), lr=CFG["lr"])
    S = torch.as_tensor(rng.standard_normal((nt, T + 1, nf)), dtype=torch.float64)
    A = torch.as_tensor(0.5 * rng.standard_normal((nt, T, a)), dtype=torch.float64)
    lengths = [T] * nt
    # neighbour table of the right shape (values irrelevant to the timing)
    I = torch.as_tensor(rng.integers(0, nt * T, (nt * T, k + 1)), dtype=torch.int64)
    D = torch.as_tensor(rng.random((nt * T, k + 1)) + 1.0, dtype=torch.float64)
    import scipy.special

    B = float(np.log(k) - scipy.special.digamma(k))
    G = float(scipy.special.gamma(d / 2 + 1))
    t = time.perf_counter()
    O.torch_policy_update(opt, beh, tgt, S, A, nt, lengths, D, I, k, G, B, d, 0.0)
    upd_s = time.perf_counter() - t
    t = time.perf_counter()
    with torch.no_grad():
        O.torch_kl(beh, tgt, S, A, nt, lengths, I, k, 0.0)
    kl_s = time.perf_counter() - t
    epoch_s = knn_s + CFG["max_off_iters"] * (upd_s + kl_s) + kl_s
    return {"value": round(epoch_s, 3), "unit": "s/epoch", "cores": cores, "kind": "port",
            "sample": (f"sklearn {sklearn.__version__} NearestNeighbors(auto, n_jobs={cores}) on "
                       f"{sample_queries} of 200000 queries x 200000 candidates (scaled x"
                       f"{X.shape[0] / sample_queries:.1f}) = {knn_s:.2f} s; one policy_update "
                       f"{upd_s:.2f} s + compute_kl {kl_s:.2f} s at full N (x30 + final H); "
                       f"torch f64 CPU, {platform.processor() or platform.machine()}")}


if __name__ == "__main__":
    main()
