"""End-to-end: the CLI runs MEPOL epochs on the GPU and writes the reference's outputs."""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env,k", [("GridWorld", 50), ("MountainCar", 4)])
def test_cli_epochs(cuda, tmp_path, env, k):
    from mepol_amd.experiments.mepol import main

    rc = main(["--env", env, "--k", str(k), "--kl_threshold", "15", "--max_off_iters", "5",
               "--learning_rate", "0.0001", "--num_trajectories", "8", "--trajectory_length", "300",
               "--num_epochs", "3", "--heatmap_every", "2", "--heatmap_episodes", "1",
               "--heatmap_num_steps", "10", "--full_entropy_traj_scale", "2", "--full_entropy_k",
               "4", "--seed", "3", "--results_dir", str(tmp_path)])
    assert rc == 0
    (run,) = glob.glob(os.path.join(tmp_path, "mepol", "*"))
    csv1 = open(os.path.join(run, f"{env}.csv")).read().strip().splitlines()
    assert csv1[0] == "epoch,loss,entropy,full_entropy,num_off_iters,execution_time"
    assert len(csv1) == 1 + 4  # epoch 0 + 3 epochs
    rows = [r.split(",") for r in csv1[1:]]
    assert [int(r[0]) for r in rows] == [0, 1, 2, 3]
    for r in rows:
        assert np.isfinite(float(r[2])) and float(r[1]) == -float(r[2])
    csv3 = open(os.path.join(run, f"{env}_off_policy_iter.csv")).read().strip().splitlines()
    assert csv3[0] == "epoch,off_policy_iter,entropy,kl,learning_rate"
    assert len(csv3) > 1
    # checkpoints at epoch 0 and every heatmap_every epochs, loadable with the safe loader
    for e in (0, 2):
        sd = torch.load(os.path.join(run, f"{e}-policy"), weights_only=True)
        assert sorted(sd) == ["log_std", "mean.bias", "mean.weight", "net.0.bias", "net.0.weight",
                              "net.2.bias", "net.2.weight"]
    assert os.path.exists(os.path.join(run, "log_info.txt"))
    # heatmap CSV (mepol.py:325-328, 247-249): epoch 0 and every heatmap_every epochs
    csv2 = open(os.path.join(run, f"{env}-heatmap.csv")).read().strip().splitlines()
    assert csv2[0] == "epoch,average_entropy"
    assert [int(r.split(",")[0]) for r in csv2[1:]] == [0, 2]
    assert all(float(r.split(",")[1]) >= 0.0 for r in csv2[1:])
