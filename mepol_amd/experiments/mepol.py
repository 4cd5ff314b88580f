"""MEPOL command line (drop-in for src/experiments/mepol.py of the reference).

Same flags, defaults and experiment specs (src/experiments/mepol.py:17-170); same results
directory layout and log_info.txt.  Runs the hot path on the GPU:

    python -m mepol_amd.experiments.mepol --env GridWorld --k 50 --kl_threshold 15 \
        --max_off_iters 30 --learning_rate 0.00001 --num_trajectories 20 \
        --trajectory_length 1200 --num_epochs 200 --heatmap_every 10 \
        --heatmap_episodes 100 --heatmap_num_steps 1200 --use_backtracking 1 \
        --zero_mean_start 1 --full_entropy_traj_scale 5 --full_entropy_k 50 --num_workers 1

MuJoCo environments (Ant, AntXY, Humanoid, HumanoidXYZ, HandReach) keep their specs but need
mujoco-py, which is outside this build's scope.  Heatmaps are computed on the GPU
(algorithms/mepol.py::get_heatmap) with the specs' discretizers.
"""
import argparse
import os
import sys
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn


def build_parser():
    p = argparse.ArgumentParser(description="MEPOL")
    p.add_argument("--num_workers", type=int, default=1,
                   help="How many parallel workers to use when collecting env trajectories and compute k-nn")
    p.add_argument("--env", type=str, required=True, help="The MDP")
    p.add_argument("--zero_mean_start", type=int, default=1, choices=[0, 1],
                   help="Whether to make the policy start from a zero mean output")
    p.add_argument("--k", type=int, required=True, help="The number of neighbors")
    p.add_argument("--kl_threshold", type=float, required=True,
                   help="The threshold after which the behavioral policy is updated")
    p.add_argument("--max_off_iters", type=int, default=20,
                   help="The maximum number of off policy optimization steps")
    p.add_argument("--use_backtracking", type=int, default=1, choices=[0, 1],
                   help="Whether to use backtracking or not")
    p.add_argument("--backtrack_coeff", type=float, default=2, help="Backtrack coefficient")
    p.add_argument("--max_backtrack_try", type=int, default=10,
                   help="Maximum number of backtracking try")
    p.add_argument("--learning_rate", type=float, required=True, help="The learning rate")
    p.add_argument("--num_trajectories", type=int, required=True,
                   help="The batch of trajectories used in off policy optimization")
    p.add_argument("--trajectory_length", type=int, required=True,
                   help="The maximum length of each trajectory in the batch of trajectories used in off policy optimization")
    p.add_argument("--num_epochs", type=int, required=True, help="The number of epochs")
    p.add_argument("--optimizer", type=str, default="adam", choices=["rmsprop", "adam"],
                   help="The optimizer")
    p.add_argument("--heatmap_every", type=int, default=10,
                   help="How many epochs to save a heatmap(if discretizer is defined)."
                        "Also the frequency at which policy weights are saved"
                        "Also the frequency at which full entropy is computed")
    p.add_argument("--heatmap_episodes", type=int, required=True,
                   help="The number of episodes on which the policy is run to compute the heatmap")
    p.add_argument("--heatmap_num_steps", type=int, required=True,
                   help="The number of steps per episode on which the policy is run to compute the heatmap")
    p.add_argument("--full_entropy_traj_scale", type=int, default=2,
                   help="The scale factor to be applied to the number of trajectories to compute the full entropy.")
    p.add_argument("--full_entropy_k", type=int, default=4,
                   help="The number of neighbors used to compute the full entropy")
    p.add_argument("--seed", type=int, default=None, help="The random seed")
    p.add_argument("--tb_dir_name", type=str, default="mepol",
                   help="The tensorboard directory under which the directory of this experiment is put")
    p.add_argument("--results_dir", type=str, default=None,
                   help="(build extension) root of results/exploration; default: ./results/exploration")
    return p


def exp_specs():
    from ..envs import ErgodicEnv, GridWorldContinuous, MountainCarContinuous
    from ..envs.discretizer import Discretizer

    xy = dict(discretizer_create=lambda env: Discretizer([[-12.0, 12.0], [-12.0, 12.0]], [40, 40],
                                                         lambda s: [s[0], s[1]]),
              heatmap_interp="spline16", heatmap_cmap="Blues", heatmap_labels=("X", "Y"))
    mujoco = dict(hidden_sizes=[400, 300], activation=nn.ReLU, log_std_init=-0.5, eps=0,
                  env_create=None)
    return {
        "MountainCar": dict(env_create=lambda: ErgodicEnv(MountainCarContinuous()),
                            discretizer_create=lambda env: Discretizer(
                                [[env.min_position, env.max_position],
                                 [-env.max_speed, env.max_speed]], [12, 11]),
                            hidden_sizes=[300, 300], activation=nn.ReLU, log_std_init=-0.5,
                            eps=1e-15, heatmap_interp="spline16", heatmap_cmap="Blues",
                            heatmap_labels=("Position", "Velocity")),
        "GridWorld": dict(env_create=lambda: ErgodicEnv(GridWorldContinuous()),
                          discretizer_create=lambda env: Discretizer(
                              [[-env.dim, env.dim], [-env.dim, env.dim]], [20, 20]),
                          hidden_sizes=[300, 300], activation=nn.ReLU, log_std_init=-1.5, eps=0,
                          heatmap_interp=None, heatmap_cmap="Blues", heatmap_labels=("X", "-Y")),
        "Ant": dict(mujoco, **xy, state_filter=list(range(7))),
        "AntXY": dict(mujoco, **xy, state_filter=list(range(2))),
        "Humanoid": dict(mujoco, **xy, state_filter=list(range(24))),
        "HumanoidXYZ": dict(mujoco, **xy, state_filter=list(range(3))),
        "HandReach": dict(mujoco, discretizer_create=lambda env: None,
                          state_filter=list(range(24))),
    }


def main(argv=None):
    from ..algorithms.mepol import mepol
    from ..policy import GaussianPolicy, train_supervised

    args = build_parser().parse_args(argv)
    specs = exp_specs()
    spec = specs.get(args.env)
    if spec is None:
        print(f"Experiment name not found. Available ones are: {', '.join(specs)}.")
        return 1
    if spec["env_create"] is None:
        print(f"{args.env} needs MuJoCo (mujoco-py), which is outside this build's scope.")
        return 2
    if not torch.cuda.is_available():
        print("mepol_amd needs a ROCm GPU (MI355X); there is no CPU path.")
        return 3
    torch.set_default_dtype(torch.float64)
    # One process per GPU under torch.distributed.run (WORLD_SIZE > 1): mepol() shards the
    # particle batch over the ranks (RCCL; gloo when ranks share a GPU).  Rank 0 picks the
    # results directory and the seed and shares them.
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        ndev = torch.cuda.device_count()
        local = int(os.environ.get("LOCAL_RANK", "0")) % ndev
        torch.cuda.set_device(local)
        dist_owned = not dist.is_initialized()
        if dist_owned:
            if ndev >= world:
                from ..parallel import prepare_nccl_env

                prepare_nccl_env()
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
        device = torch.device("cuda", local)
    else:
        device = torch.device("cuda")
    rank = dist.get_rank() if dist is not None else 0
    env = spec["env_create"]()
    state_filter = spec.get("state_filter")
    eps = spec["eps"]

    def create_policy(is_behavioral=False):
        policy = GaussianPolicy(num_features=env.num_features, hidden_sizes=spec["hidden_sizes"],
                                action_dim=env.action_space.shape[0],
                                activation=spec["activation"],
                                log_std_init=spec["log_std_init"]).to(device)
        if is_behavioral and args.zero_mean_start:
            policy = train_supervised(env, policy, train_steps=100, batch_size=5000)
        return policy

    exp_name = (f"env={args.env},z_mu_start={args.zero_mean_start},k={args.k},"
                f"kl_thresh={args.kl_threshold},max_off_iters={args.max_off_iters},"
                f"num_traj={args.num_trajectories},traj_len={args.trajectory_length},"
                f"lr={args.learning_rate},opt={args.optimizer},"
                f"fe_traj_sc={args.full_entropy_traj_scale},fe_k={args.full_entropy_k},"
                f"use_bt={args.use_backtracking},bt_coeff={args.backtrack_coeff},"
                f"max_bt_try={args.max_backtrack_try}")
    root = args.results_dir or os.path.join(os.getcwd(), "results", "exploration")
    out_path = os.path.join(root, args.tb_dir_name, exp_name + "__" +
                            datetime.now().strftime("%Y_%m_%d_%H_%M_%S") + "__" + str(os.getpid()))
    if rank == 0:
        os.makedirs(out_path, exist_ok=True)
    with open(os.path.join(out_path, "log_info.txt") if rank == 0 else os.devnull, "w") as f:
        f.write("Run info:\n")
        f.write("-" * 10 + "\n")
        for key, value in vars(args).items():
            f.write(f"{key}={value}\n")
        f.write("-" * 10 + "\n")
        f.write(str(create_policy()))
        f.write("\n")
        if args.seed is None:
            args.seed = int(np.random.randint(2 ** 16 - 1))
            f.write(f"Setting random seed {args.seed}\n")
    if dist is not None:
        shared = [out_path, args.seed]
        dist.broadcast_object_list(shared, src=0)
        out_path, args.seed = shared

    mepol(env=env, env_name=args.env, state_filter=state_filter, create_policy=create_policy,
          k=args.k, kl_threshold=args.kl_threshold, max_off_iters=args.max_off_iters,
          use_backtracking=args.use_backtracking, backtrack_coeff=args.backtrack_coeff,
          max_backtrack_try=args.max_backtrack_try, eps=eps, learning_rate=args.learning_rate,
          num_traj=args.num_trajectories, traj_len=args.trajectory_length,
          num_epochs=args.num_epochs, optimizer=args.optimizer,
          full_entropy_traj_scale=args.full_entropy_traj_scale,
          full_entropy_k=args.full_entropy_k, heatmap_every=args.heatmap_every,
          heatmap_discretizer=spec["discretizer_create"](env),
          heatmap_episodes=args.heatmap_episodes, heatmap_num_steps=args.heatmap_num_steps,
          heatmap_cmap=spec.get("heatmap_cmap"), heatmap_labels=spec.get("heatmap_labels"),
          heatmap_interp=spec.get("heatmap_interp"), seed=args.seed, out_path=out_path,
          num_workers=args.num_workers)
    if dist is not None:
        dist.barrier()
        if dist_owned:
            from ..parallel import destroy_process_group

            destroy_process_group(dist)
    return 0


if __name__ == "__main__":
    sys.exit(main())
