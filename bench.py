"""MEPOL epoch benchmark on MI355X (BASELINE.json metric: epoch wall-clock + k-NN roofline).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C2|C2S|C3|C4|C5]

Workloads (BASELINE.json configs):
  C3  (default) Ant-shaped batch: N = 400 x 500 = 200,000 particles, k-NN space d = 29, k = 30,
      policy 29 -> [400, 300] -> 8 (f64, as the reference), Adam lr 1e-5, KL threshold 15,
      30 off-policy iterations.  MuJoCo is out of scope, so the rollout is replaced by a seeded
      synthetic batch resident in HBM (states ~ N(0,1) f32, actions ~ N(0, 0.5^2) f32); one
      step = one epoch of the reference's timed window (mepol.py:405 -> 499) minus the rollout:
      exact k-NN + off-policy loop (policy_update + compute_kl until the stop rule) + final H.
  C4  Humanoid-shaped: N = 200,000, d = 47, k = 30, policy 47 -> [400, 300] -> 17.
  C5  HandReach-shaped: N = 10,000 x 50 = 500,000, d = 63, k = 50, policy 63 -> [400, 300] -> 20.
  C2  GridWorld, the whole epoch window including the rollout on the GPU: 20 x 1000 = 20,000
      particles, k = 4 (BASELINE config), policy 2 -> [300, 300] -> 2, log_std -1.5.
  C2S GridWorld at the reference script's settings (scripts/tae/grid_world.sh): 20 x 1200 =
      24,000 particles, k = 50 -- the configuration SURVEY §6 timed at 9.10 s per epoch.

Multi-GPU: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) each process is a
rank; `--gpus N` without a launcher spawns the N ranks itself (fresh child processes, before
any GPU call in the parent).  Rank r owns trajectories [r nt/N, (r+1) nt/N); next states are
all-gathered (RCCL over xGMI) before the k-NN, each rank answers its own queries, and the
per-iteration scalars / weight vectors / parameter gradients are reduced so every rank takes the
same steps (strong scaling: fixed N).  With fewer GPUs than ranks the ranks share the GPUs over
gloo and the line says "rehearsal".
"""
import argparse
import json
import os
import platform
import socket
import subprocess
import sys
import time

import numpy as np

COMMON = dict(max_off_iters=30, backtrack_coeff=2, max_backtrack_try=10, lr=1e-5,
              kl_threshold=15.0, eps=0.0, log_std_init=-0.5)
WORKLOADS = {
    "C3": dict(COMMON, num_traj=400, traj_len=500, nf=29, a=8, hidden=[400, 300], k=30, d=29,
               name="C3 Ant-shaped MEPOL epoch (k-NN + off-policy loop + final H)"),
    "C4": dict(COMMON, num_traj=400, traj_len=500, nf=47, a=17, hidden=[400, 300], k=30, d=47,
               name="C4 Humanoid-shaped MEPOL epoch (k-NN + off-policy loop + final H)"),
    "C5": dict(COMMON, num_traj=10000, traj_len=50, nf=63, a=20, hidden=[400, 300], k=50, d=63,
               name="C5 HandReach-shaped MEPOL epoch (k-NN + off-policy loop + final H)"),
    # Rank 0 of the 8-GPU strong-scaling run, emulated on one GPU (_EmulatedDist): its 1/8 of
    # the particles through the sharded code path (ShardedEpoch + ShardedIteration), the k-NN of
    # its queries against ALL N candidates, every collective replaced by local copies of the
    # same size (no peers, no xGMI): the per-rank compute of C3/C4/C5 at 8 GPUs.
    "C3R8": dict(COMMON, num_traj=400, traj_len=500, nf=29, a=8, hidden=[400, 300], k=30, d=29,
                 emulate_world=8,
                 name="C3 rank-0 share at 8 GPUs (25k of 200k particles; k-NN vs all 200k)"),
    "C4R8": dict(COMMON, num_traj=400, traj_len=500, nf=47, a=17, hidden=[400, 300], k=30, d=47,
                 emulate_world=8,
                 name="C4 rank-0 share at 8 GPUs (25k of 200k particles; k-NN vs all 200k)"),
    "C5R8": dict(COMMON, num_traj=10000, traj_len=50, nf=63, a=20, hidden=[400, 300], k=50,
                 d=63, emulate_world=8,
                 name="C5 rank-0 share at 8 GPUs (62.5k of 500k particles; k-NN vs all 500k)"),
    "C2": dict(COMMON, num_traj=20, traj_len=1000, nf=2, a=2, hidden=[300, 300], k=4, d=2,
               log_std_init=-1.5, env="GridWorld",
               name="C2 GridWorld MEPOL epoch (GPU rollout + k-NN + off-policy loop + final H)"),
    "C2S": dict(COMMON, num_traj=20, traj_len=1200, nf=2, a=2, hidden=[300, 300], k=50, d=2,
                log_std_init=-1.5, env="GridWorld",
                name="C2S GridWorld MEPOL epoch at scripts/tae/grid_world.sh settings "
                     "(GPU rollout + k-NN + off-policy loop + final H)"),
}
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector == FP32 matrix peak
PEAK_F16_TFLOPS = 2500.0   # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense
PEAK_HBM_GBPS = 8000.0
ROOT = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", default="C3", choices=sorted(WORKLOADS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample-queries", type=int, default=16000)
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the live rocprofv3 --pmc passes for roofline.traffic (the stamped "
                        "profiles/knn_pmc_<workload>.json is read instead)")
    p.add_argument("--selftest", action="store_true",
                   help="launcher plumbing only (no GPU): ranks rendezvous over gloo, time an "
                        "empty step with the max-over-ranks clock and print the JSON line")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# launcher: --gpus N without torch.distributed.run
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn(args, argv):
    """Start args.gpus rank processes (this file, same flags) and wait for them.  Runs before
    any GPU call in this process (device_count does not initialise the GPU on this image)."""
    import torch

    n = args.gpus
    ndev = torch.cuda.device_count()
    backend = "nccl" if ndev >= n and not args.selftest else "gloo"
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   MEPOL_BENCH_BACKEND=backend, MEPOL_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


# ---------------------------------------------------------------------------------------------
# the benchmark proper (one rank)
# ---------------------------------------------------------------------------------------------
def synthetic_batch(cfg, seed, device, rank=0, world=1):
    import torch

    g = torch.Generator(device=device).manual_seed(seed)
    nt, T, nf, a = cfg["num_traj"], cfg["traj_len"], cfg["nf"], cfg["a"]
    per = nt // world
    states = torch.randn((nt, T + 1, nf), generator=g, device=device, dtype=torch.float32)
    actions = 0.5 * torch.randn((nt, T, a), generator=g, device=device, dtype=torch.float32)
    return (states[rank * per:(rank + 1) * per].contiguous(),
            actions[rank * per:(rank + 1) * per].contiguous())


class _EmulatedDist:
    """Rank 0 of a `world`-rank job on one GPU, without peers: the torch.distributed calls that
    ShardedEpoch / ShardedIteration make, each replaced by local copies of the same size.
    all_gather_into_tensor fills the peers' slots from `peers` (a list of world - 1 tensors)
    when one of that shape and dtype is registered -- the other shards' next states, so the
    k-NN runs against the full candidate set -- and with rank 0's own payload otherwise;
    all_reduce keeps rank 0's values (one in-place pass over the payload).  Per-rank compute of the multi-GPU run, not its result."""

    class ReduceOp:
        SUM, MIN, MAX = "sum", "min", "max"

    def __init__(self, world):
        self.world = world
        self.peers = []

    def get_world_size(self, group=None):
        return self.world

    def get_rank(self, group=None):
        return 0

    def get_backend(self, group=None):
        return "nccl"  # the graph path captures these copies like RCCL collectives

    def all_gather_into_tensor(self, out, inp, group=None):
        o = out.view(self.world, -1)
        flat = inp.reshape(-1)
        pe = self.peers  # ShardedEpoch gathers flattened tensors: match by size and dtype
        if not (pe and pe[0].numel() == inp.numel() and pe[0].dtype == inp.dtype):
            # one launch writing all world slots, as RCCL's one all_gather kernel does
            o.copy_(flat.unsqueeze(0).expand(self.world, -1))
            return
        o[0].copy_(flat)
        for r in range(1, self.world):
            o[r].copy_(pe[r - 1].reshape(-1))

    def all_reduce(self, t, op=None, group=None):
        # a device pass over the same payload in place (x * 1 is exact, any dtype): one launch that reads
        # and writes the bytes, a lower bound for RCCL's reduce-scatter + all-gather (the xGMI
        # cost model is DESIGN.md section 6)
        t.mul_(1)


def selftest(args):
    """The multi-rank launch path without a GPU: rendezvous, barrier, max-over-ranks timing."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    x = torch.full((1,), float(rank + 1), dtype=torch.float64)
    for _ in range(args.steps):
        if world > 1:
            dist.all_reduce(x)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
    if rank == 0:
        print(json.dumps({"metric": "bench launcher selftest", "value": elapsed, "unit": "s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "selftest": True, "sum_of_ranks": float(x.item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


_JSON_FD = None


def _quiet_stdout():
    """Route fd 1 to /dev/null for the rest of the run and keep the real stdout for the one
    JSON line: RCCL prints its version banner on stdout when a communicator is created, and the
    contract is a single JSON line from rank 0."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)
        os.close(null)


def _emit(line):
    text = json.dumps(line) + "\n"
    if _JSON_FD is None:
        print(text, end="", flush=True)
    else:
        sys.stdout.flush()
        os.write(_JSON_FD, text.encode())


def run(args):
    import torch

    if args.selftest:
        return selftest(args)
    cfg = WORKLOADS[args.workload]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    ndev = max(torch.cuda.device_count(), 1)
    local = int(os.environ.get("LOCAL_RANK", "0")) % ndev
    if world > 1 and args.gpus != world and rank == 0:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE",
              file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    backend = None
    # MEPOL_BENCH_SHARDED=1 runs the multi-rank code path (ShardedEpoch + captured RCCL
    # collectives) at world size 1: a one-GPU rehearsal of what --gpus N runs per rank.
    sharded = world > 1 or os.environ.get("MEPOL_BENCH_SHARDED") == "1"
    emul = None
    if cfg.get("emulate_world"):
        if world > 1:
            raise SystemExit(f"bench: {args.workload} emulates one rank of "
                             f"{cfg['emulate_world']} on one GPU; run it with --gpus 1")
        emul = _EmulatedDist(cfg["emulate_world"])
        sharded = True
    if sharded and emul is None:
        import torch.distributed as dist

        _quiet_stdout()

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        backend = os.environ.get("MEPOL_BENCH_BACKEND", "nccl")  # nccl == RCCL on ROCm
        if backend == "nccl":
            from mepol_amd.parallel import prepare_nccl_env

            prepare_nccl_env()
            dist.init_process_group("nccl", device_id=dev)
        else:  # rehearsal: several ranks share one GPU over gloo
            dist.init_process_group(backend)
    import scipy.special

    from mepol_amd.algorithms import mepol as M
    from mepol_amd.policy import GaussianPolicy

    k, nf, a, d = cfg["k"], cfg["nf"], cfg["a"], cfg["d"]
    nt, T = cfg["num_traj"], cfg["traj_len"]
    shards = emul.world if emul is not None else world   # ranks the particles are split over
    if nt % shards:
        raise SystemExit(f"bench: {nt} trajectories do not split over {shards} ranks")
    ns = d
    B = float(np.log(k) - scipy.special.digamma(k))
    G = float(scipy.special.gamma(ns / 2 + 1))
    rollout = cfg.get("env") is not None
    torch.manual_seed(0)
    env = None
    if rollout:
        from mepol_amd.envs import ErgodicEnv, GridWorldContinuous
        from mepol_amd.policy import train_supervised

        env = ErgodicEnv(GridWorldContinuous())
        behavioral = GaussianPolicy(cfg["hidden"], nf, a, cfg["log_std_init"]).to(dev)
        train_supervised(env, behavioral, 100, 5000)  # --zero_mean_start 1 (outside the window)
        torch.cuda.manual_seed(1000 + rank)  # independent rollout noise / resets per rank
    else:
        behavioral = GaussianPolicy(cfg["hidden"], nf, a, cfg["log_std_init"]).to(dev)
    target = GaussianPolicy(cfg["hidden"], nf, a, cfg["log_std_init"]).to(dev)
    last_valid = GaussianPolicy(cfg["hidden"], nf, a, cfg["log_std_init"]).to(dev)
    target.load_state_dict(behavioral.state_dict())
    last_valid.load_state_dict(behavioral.state_dict())
    opt = torch.optim.Adam(target.parameters(), lr=cfg["lr"])
    N = nt * T

    batches = [] if rollout else [synthetic_batch(cfg, s, dev, rank, shards) for s in range(3)]
    peers = []  # emulation: the other shards' next states of each batch (k-NN candidates)
    if emul is not None:
        for s_ in range(3):
            peers.append([synthetic_batch(cfg, s_, dev, r, shards)[0][:, 1:].reshape(-1, nf)
                          [:, :d].contiguous() for r in range(1, shards)])
    knn_events, roll_events, iters_done, entropies = [], [], [], []

    def one_epoch(i):
        T_ = T
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e2 = torch.cuda.Event(enable_timing=True)
        last_valid.load_state_dict(behavioral.state_dict())
        e0.record()
        if rollout:
            st32, ac32, rtl32, nxt = M.collect_particles_device(env, behavioral, nt // world, T_,
                                                                None)
            nt_local = nt // world
        else:
            st32, ac32 = batches[i % len(batches)]
            nt_local = st32.shape[0]
            nxt = st32[:, 1:].reshape(-1, nf)[:, :d].contiguous()
        e1.record()
        st = st32.double()
        ac = ac32.double()
        rtl = torch.full((nt_local, 1), T_, dtype=torch.int64, device=dev)
        if not sharded:
            # the k-NN call alone is timed (the roofline line); the batch set-up and CSR build
            # after it are inside the epoch, not inside knn_ms
            k0 = torch.cuda.Event(enable_timing=True)
            k1 = torch.cuda.Event(enable_timing=True)
            st_, ac_, rl_, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, k,
                                                           knn_events=(k0, k1))
            e2.record()
            res = M.off_policy_optimization(
                opt, behavioral, target, last_valid, st_, ac_, nt_local, rl_, D, I, k, G, B, ns,
                cfg["eps"], cfg["kl_threshold"], cfg["max_off_iters"], True,
                cfg["backtrack_coeff"], cfg["max_backtrack_try"], cfg["lr"])
        else:
            from mepol_amd.parallel import ShardedEpoch

            if emul is not None:
                emul.peers = peers[i % len(peers)]
            ep = ShardedEpoch(st, ac, rtl, nxt, k, emul if emul is not None else dist)
            ep.build_knn()
            e2.record()
            res = ep.off_policy_optimization(
                opt, behavioral, target, last_valid, G, B, ns, cfg["eps"], cfg["kl_threshold"],
                cfg["max_off_iters"], True, cfg["backtrack_coeff"], cfg["max_backtrack_try"],
                cfg["lr"])
        entropy, n_off, _, _ = res
        behavioral.load_state_dict(last_valid.state_dict())
        target.load_state_dict(last_valid.state_dict())
        entropies.append(float(entropy))
        roll_events.append((e0, e1))
        knn_events.append((k0, k1) if not sharded else (e1, e2))
        iters_done.append(n_off)

    for i in range(args.warmup):
        one_epoch(i)
    for lst in (knn_events, roll_events, iters_done, entropies):
        lst.clear()
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
    knn_ms = float(np.mean([x.elapsed_time(y) for x, y in knn_events]))
    roll_ms = float(np.mean([x.elapsed_time(y) for x, y in roll_events]))
    per_rank_knn = [knn_ms]
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        kt = torch.tensor([knn_ms], device=dev, dtype=torch.float64)
        allk = [torch.zeros_like(kt) for _ in range(world)]
        dist.all_gather(allk, kt)
        per_rank_knn = [float(x.item()) for x in allk]
    epoch_s = elapsed / args.steps

    if rank != 0:
        if dist is not None:
            from mepol_amd import parallel

            parallel.destroy_process_group(dist)
        return

    from mepol_amd import parallel
    from mepol_amd.algorithms import device_loop

    it = (parallel._SHARDED_CACHE if sharded else device_loop._CACHE).get(target)
    iteration_path = "hip-graph replay" if it is not None and it.graph is not None else "eager"
    nq = N // shards
    F = 3.0 * d * nq * N                      # algorithmic flops
    knn_tflops = F / (knn_ms * 1e-3) / 1e12
    # The selection (csrc/knn.hip, make_plan): f16 MFMA with the candidates' hi half (nh = 1:
    # 1 product per k-step at <= 3 k-steps, q_lo added at 4) or hi + lo halves (nh = 2, 3
    # products), 2 x K flops each per (query, candidate) tile pair, K = 16*ceil((d+1)/16), f32
    # accumulate; then the certified f64 refine.
    from mepol_amd import ops as _ops

    plan = _ops.knn_plan(N, nq, d, k + 1)
    knn_issued = _ops.knn_issued_mfma_flops(N, nq, plan)
    knn_peak = PEAK_F16_TFLOPS
    knn_desc = (("f16 MFMA selection (candidate hi half x split query" if plan["nh"] == 1 else
                 "f16 MFMA selection (split candidate x split query, 3 products")
                + ", f32 accumulate) + certified f64 exact refine (bit-exact output)")
    traffic, traffic_note, traffic_kernels = None, None, None
    live = getattr(args, "live_traffic", None)
    pmc_path = os.path.join(ROOT, "profiles", f"knn_pmc_{args.workload}.json")
    if live is not None and live[0] is not None:
        traffic, traffic_kernels = live[0], live[1]
    elif os.path.exists(pmc_path) and world == 1 and emul is None:
        # counters were taken on the 1-GPU k-NN call
        # the PMC passes (tools/knn_pmc.sh -> tools/knn_pmc_summary.py) stamp the file with a
        # hash of the k-NN sources they measured; a file from other sources is not reported
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("knn_source_stamp") == knn_source_stamp():
                traffic = pmc.get("hbm_bytes_per_launch")
            else:
                traffic_note = (f"{os.path.relpath(pmc_path, ROOT)} was measured on other k-NN "
                                "sources (stamp mismatch): not reported")
        except Exception as e:
            traffic_note = f"unreadable {pmc_path}: {e!r}"
    rehearsal = sharded and backend != "nccl" and world > 1
    line = {
        "metric": f"MEPOL epoch wall-clock ({args.workload}: N={N}, d={d}, k={k}"
                  + ("; rollout included)" if rollout else "; rollout excluded)"),
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
        "data": "synthetic" if not rollout else "GridWorld rollouts of a random-init policy",
        "config": {"workload": cfg["name"], "particles": N, "num_traj": nt, "traj_len": T,
                   "d": d, "k": k, "policy": f"{nf}->{cfg['hidden']}->{a} f64",
                   "off_policy_iters": float(np.mean(iters_done)),
                   "parallelism": (f"rank 0 of dp{shards} emulated on 1 GPU (collectives -> local "
                                   f"copies of the same size)" if emul is not None
                                   else f"dp{world}"),
                   "knn_precision": knn_desc, "off_policy_iteration": iteration_path},
        "particles_per_s": round(N / shards / epoch_s, 1),
        "knn_ms": round(knn_ms, 3),
        "knn_ms_per_rank": [round(x, 3) for x in per_rank_knn],
        "roofline": {"bound": "mfma", "achieved": round(knn_tflops, 2), "peak": knn_peak,
                     "unit": "TFLOP/s", "frac": round(knn_tflops / knn_peak, 4),
                     "mfma_issued_tflops": round(knn_issued / (knn_ms * 1e-3) / 1e12, 2),
                     "mfma_issued_frac": round(knn_issued / (knn_ms * 1e-3) / 1e12 / knn_peak, 4),
                     "mfma_products_per_kstep": plan["mfma_products"],
                     "traffic": traffic,
                     "kernel": ("k-NN call (norms + pack + select + refine + exact), HIP events "
                                "around the call on its launch stream" if not sharded else
                                "k-NN phase of the sharded epoch (candidate all-gather + k-NN "
                                "call + index all-gather + CSR build), HIP events")
                               + "; achieved = F/t, F = 3*d*Nq*Nc (SURVEY 8d)"},
    }
    if live is not None and live[0] is None:
        traffic_note = f"live PMC passes failed ({live[2]})" + (
            f"; {traffic_note}" if traffic_note else
            (f"; reported from {os.path.relpath(pmc_path, ROOT)}" if traffic else ""))
    if traffic_note:
        line["roofline"]["traffic_note"] = traffic_note
    if traffic and traffic_kernels is not None:
        line["roofline"]["traffic_source"] = (
            "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (one counter each) over "
            "tools/knn_probe.py at this shape, run by this bench before it touched the GPU; "
            "FETCH_SIZE x2 (gfx950)")
        line["roofline"]["traffic_per_kernel"] = traffic_kernels
        comp = 4 * d * (nq + N) + 8 * (k + 1) * nq
        line["roofline"]["traffic_compulsory"] = comp
        line["roofline"]["traffic_over_compulsory"] = round(traffic / comp, 2)
    elif traffic:
        line["roofline"]["traffic_source"] = os.path.relpath(pmc_path, ROOT)
    if traffic:
        # BASELINE's literal metric ("k-NN HBM GB/s, % of 8 TB/s"): the measured HBM bytes per
        # call over the call's time.  The candidates stay in L2 / MALL, so this is far from the
        # bound the call runs against (roofline.bound: the f16 MFMA peak)
        gbps = traffic / (knn_ms * 1e-3) / 1e9
        line["roofline"]["hbm_GBps"] = round(gbps, 1)
        line["roofline"]["hbm_frac"] = round(gbps / PEAK_HBM_GBPS, 4)
    mlp = _mlp_roofline(it) if (it is not None and not sharded) else None
    if mlp:
        line["roofline_iteration"] = mlp
    if rollout:
        line["rollout_ms"] = round(roll_ms, 3)
        line["rollout_us_per_step"] = round(roll_ms * 1e3 / T, 2)
        line["final_entropy"] = float(np.mean(entropies))
        line["survey_reference_epoch_s"] = 9.10 if args.workload == "C2S" else None
    if rehearsal:
        line["config"]["rehearsal"] = f"{world} ranks on {torch.cuda.device_count()} GPU(s), gloo"
    if not args.no_cpu_baseline and world == 1 and emul is None:
        line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_sample_queries, iters_done)
    _emit(line)
    if dist is not None:
        parallel.destroy_process_group(dist)


def knn_source_stamp():
    """Hash of the k-NN sources (csrc/knn*.hip / *.hpp): ties a PMC traffic file to the code it
    was measured on (the GPU box has the sources but no git history)."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "mepol_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if f.startswith("knn") or f == "common.hpp":
            h.update(f.encode())
            h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()[:16]


PEAK_F64_TFLOPS = 78.6            # MI355X spec: FP64 matrix (dense)
MEASURED_F64_MFMA_TFLOPS = 77.9   # tools/f64_mfma_table.hip (profiles/r5/f64/): 16x16x4, >= 2 waves/SIMD


def _mlp_roofline(it):
    """The iteration's two MFMA kernels timed on their own after the timed region (inside the
    replayed graph they cannot be event-timed): the fused forward (csrc/policy_fwd.hip) and the
    fused dh1 GEMM + layer-1 backward (csrc/gemm.hip), on the device iteration's own buffers."""
    import torch

    from mepol_amd import ops

    if not getattr(it, "fused_fwd", False) or not getattr(it, "fused_dh1", False):
        return None
    W1, b1, W2, b2, Wm, bm, ls = it.named
    N, F = it.x.shape
    h0, h1w = W1.shape[0], W2.shape[0]
    dz2 = torch.randn(N, h1w, dtype=torch.float64, device=it.x.device)
    W2t = W2.detach().t().contiguous()
    reps = 5

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e-3

    with torch.no_grad():
        t_f = timed(lambda: ops.policy_forward(it.x, W1, b1, W2, b2, Wm, bm, ls, it.act, it.h1,
                                               it.z2, it.mu, it.logp,
                                               mask_out=getattr(it, "h1_mask", None)))
        t_b = timed(lambda: ops.dh1_layer1_backward(dz2, W2t, it.h1, it.x, ws=it.ws_dh1,
                                                    mask=getattr(it, "h1_mask", None)))
    fl_f = 2.0 * N * (h0 * h1w + F * h0)
    fl_b = 2.0 * N * (h1w * h0 + h0 * (F + 1))
    out = {"bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_F64_TFLOPS,
           "measured_f64_mfma_ceiling": MEASURED_F64_MFMA_TFLOPS, "traffic": None,
           "note": "f64 MFMA kernels of the off-policy iteration, each timed alone with HIP "
                   "events after the timed region; achieved = algorithmic flops / time"}
    for key, t, fl in (("policy_forward", t_f, fl_f), ("dh1_layer1_backward", t_b, fl_b)):
        out[key] = {"us": round(t * 1e6, 1), "achieved": round(fl / t / 1e12, 2),
                    "frac": round(fl / t / 1e12 / PEAK_F64_TFLOPS, 4)}
    return out


# ---------------------------------------------------------------------------------------------
# CPU baseline: the oracle (reference-shaped CPU restatement) on the host cores
# ---------------------------------------------------------------------------------------------
def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _cpu_threads():
    """Host threads for the baseline: the CPUs this process may run on, capped by the box's
    declared share (OMP_NUM_THREADS is set to it on the GPU box)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(aff, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else aff), aff


def cpu_baseline(cfg, sample_queries, iters_done):
    """Bounded sample of one epoch on the oracle (torch f64 + sklearn, reference-shaped):
    sklearn k-NN for `sample_queries` queries against all candidates (scaled to N queries), one
    policy_update + one compute_kl at full N (scaled by the GPU run's iteration count) plus the
    final entropy, and for rollout workloads the reference's per-step batch-1 rollout over two
    trajectories (scaled to num_traj)."""
    import torch
    import scipy.special
    import sklearn
    from sklearn.neighbors import NearestNeighbors

    from oracle import mepol_oracle as O

    cores, aff = _cpu_threads()
    torch.set_num_threads(cores)
    k, nf, a, d = cfg["k"], cfg["nf"], cfg["a"], cfg["d"]
    nt, T = cfg["num_traj"], cfg["traj_len"]
    N = nt * T
    rng = np.random.default_rng(0)
    torch.manual_seed(0)
    beh = O.TorchPolicy(cfg["hidden"], nf, a, cfg["log_std_init"])
    tgt = O.TorchPolicy(cfg["hidden"], nf, a, cfg["log_std_init"])
    tgt.load_state_dict(beh.state_dict())
    roll_s = 0.0
    if cfg.get("env") in ("GridWorld", "MountainCar"):
        # collect_particles (mepol.py:76-109): batch-1 policy.predict + env.step per step
        nsamp = 2
        mc = cfg["env"] == "MountainCar"
        if mc:
            step, reset = O.mountaincar_step_scalar, lambda: np.array([rng.uniform(-0.6, -0.4), 0.0])
        else:
            step, reset = O.gridworld_step_scalar, lambda: rng.uniform(-6, -4, 2).astype(np.float32)
        t = time.perf_counter()
        O.collect_particles_scalar(step, reset, beh, nsamp, T, nf, a)
        roll_s = (time.perf_counter() - t) * nt / nsamp
        lo, hi = ((-1.2, 0.6) if mc else (-6, 6))
        X = rng.uniform(lo, hi, (N, d)).astype(np.float32)
    else:
        X = rng.standard_normal((N, d)).astype(np.float32)
    nq = min(sample_queries, N)
    t = time.perf_counter()
    nbrs = NearestNeighbors(n_neighbors=k + 1, metric="euclidean", algorithm="auto", n_jobs=cores)
    nbrs.fit(X)
    nbrs.kneighbors(X[:nq])
    knn_s = (time.perf_counter() - t) * (N / nq)
    opt = torch.optim.Adam(tgt.parameters(), lr=cfg["lr"])
    S = torch.as_tensor(rng.standard_normal((nt, T + 1, nf)), dtype=torch.float64)
    A = torch.as_tensor(0.5 * rng.standard_normal((nt, T, a)), dtype=torch.float64)
    lengths = [T] * nt
    # neighbour table of the right shape (values irrelevant to the timing)
    I = torch.as_tensor(rng.integers(0, N, (N, k + 1)), dtype=torch.int64)
    D = torch.as_tensor(rng.random((N, k + 1)) + 1.0, dtype=torch.float64)
    B = float(np.log(k) - scipy.special.digamma(k))
    G = float(scipy.special.gamma(d / 2 + 1))
    t = time.perf_counter()
    O.torch_policy_update(opt, beh, tgt, S, A, nt, lengths, D, I, k, G, B, d, 0.0)
    upd_s = time.perf_counter() - t
    t = time.perf_counter()
    with torch.no_grad():
        O.torch_kl(beh, tgt, S, A, nt, lengths, I, k, 0.0)
    kl_s = time.perf_counter() - t
    iters = float(np.mean(iters_done)) if iters_done else float(cfg["max_off_iters"])
    epoch_s = roll_s + knn_s + iters * (upd_s + kl_s) + kl_s
    algo = nbrs._fit_method  # what 'auto' chose here (brute above d = 15 in sklearn >= 1.x)
    sample = (f"sklearn {sklearn.__version__} NearestNeighbors(auto -> {algo}, n_jobs={cores}) on "
              f"{nq} of {N} queries x {N} candidates (scaled x{N / nq:.1f}) = {knn_s:.2f} s "
              f"(generous to the CPU where 'auto' picks brute: the reference pins sklearn 0.22, "
              f"whose 'auto' picks kd_tree, far slower in high d); one "
              f"policy_update {upd_s:.2f} s + compute_kl {kl_s:.2f} s at full N "
              f"(x{iters:g} + final H)")
    if roll_s:
        sample += f"; batch-1 rollout of 2 of {nt} trajectories x {T} steps (scaled) = {roll_s:.2f} s"
    cal = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    ratio = None
    if os.path.exists(cal):
        try:
            ratio = json.load(open(cal)).get("epoch_ratio_summary")
        except Exception:
            ratio = None
    return {"value": round(epoch_s, 3), "unit": "s/epoch", "cores": cores, "kind": "port",
            "sample": sample + "; torch f64 CPU", "cpu_model": _cpu_model(),
            "affinity_cpus": aff,
            # SURVEY 8(d) asks for all affinity CPUs; the box's declared CPU share is
            # OMP_NUM_THREADS (16 per GPU), which the harness asks worker pools to respect.  The
            # measured value uses the share; this is the same epoch at perfect scaling to every
            # affinity CPU (a lower bound on the CPU time there), so the GPU/CPU ratio lies
            # between the two.
            "value_ideal_at_affinity": round(epoch_s * cores / aff, 3),
            "components_s": {"rollout": round(roll_s, 3), "knn": round(knn_s, 3),
                             "policy_update": round(upd_s, 3), "compute_kl": round(kl_s, 3),
                             "iterations": iters},
            "calibration_vs_reference": ratio}


def _under_profiler():
    return ("rocprof" in os.environ.get("LD_PRELOAD", "")
            or any(k.startswith("ROCPROF") for k in os.environ))


def live_knn_traffic(cfg):
    """HBM bytes of one k-NN call at this workload's shape, measured in THIS bench run: two
    rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: one counter per pass, as MI355X_MICROARCH.md
    prescribes) over tools/knn_probe.py as child processes, started before this process touches
    the GPU.  FETCH_SIZE is doubled (gfx950), WRITE_SIZE taken as reported (tools/knn_pmc_summary).
    Returns (bytes, per-kernel dict, note) or (None, None, reason)."""
    import shutil
    import signal
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, None, "rocprofv3 not on PATH"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from knn_pmc_summary import per_call

    N, d, k = cfg["num_traj"] * cfg["traj_len"], cfg["d"], cfg["k"]
    out = tempfile.mkdtemp(prefix="mepol_pmc_", dir="/tmp")
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        cmd = [prof, "--pmc", c, "-d", os.path.join(out, c), "-o", "run", "--", sys.executable,
               os.path.join(ROOT, "tools", "knn_probe.py"), "--n", str(N), "--d", str(d),
               "--kp1", str(k + 1), "--reps", "1"]
        p = subprocess.Popen(cmd, cwd="/tmp", env=dict(os.environ, TMPDIR="/tmp"),
                             stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                             start_new_session=True)
        try:
            rc = p.wait(timeout=150)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.wait()
            return None, None, f"rocprofv3 --pmc {c} pass timed out"
        if rc != 0:
            return None, None, f"rocprofv3 --pmc {c} pass exited {rc}"
        try:
            res[c] = per_call(os.path.join(out, c, "run_results.db"), c)
        except Exception as e:  # no database / no k-NN dispatch in it
            return None, None, f"rocprofv3 --pmc {c} output unreadable: {e!r}"
    shutil.rmtree(out, ignore_errors=True)
    fetch, write = res["FETCH_SIZE"], res["WRITE_SIZE"]
    kernels = {kk.split("::")[-1][:60]: {"fetch_x2": round(2 * fetch.get(kk, 0.0)),
                                          "write": round(write.get(kk, 0.0))}
               for kk in sorted(set(fetch) | set(write))}
    total = sum(2 * v for v in fetch.values()) + sum(write.values())
    return total, kernels, None


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn(args, argv)
    cfg = WORKLOADS[args.workload]
    args.live_traffic = None
    if (not args.no_pmc and not args.selftest and "WORLD_SIZE" not in os.environ
            and cfg.get("env") is None and not cfg.get("emulate_world")):
        if _under_profiler():
            args.live_traffic = (None, None, "bench runs under a profiler: live PMC passes skipped")
        else:  # before this process makes any GPU call
            args.live_traffic = live_knn_traffic(cfg)
    run(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
