"""The drop-in CLI / mepol() in multi-rank mode: two ranks (one process each,
sharing the box's GPU over gloo) reproduce the one-rank run's CSV rows.  The rollout draws the
noise of every trajectory up front, so the ranks' shards concatenate to the one-rank batch;
ShardedEpoch keeps H, KL and the parameters identical on every rank."""
import glob
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--env", "MountainCar", "--k", "4", "--kl_threshold", "15", "--max_off_iters", "4",
        "--learning_rate", "0.0001", "--num_trajectories", "8", "--trajectory_length", "400",
        "--num_epochs", "2", "--heatmap_every", "2", "--heatmap_episodes", "2",
        "--heatmap_num_steps", "20", "--full_entropy_traj_scale", "2", "--full_entropy_k", "4",
        "--seed", "11"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, out):
    base = {k: v for k, v in os.environ.items()
            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    port = str(_port())
    procs = []
    for r in range(world):
        env = dict(base, PYTHONPATH=ROOT)
        if world > 1:
            env.update(WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(r),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "mepol_amd.experiments.mepol"] + ARGS + ["--results_dir", out],
            env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-3000:] for o in outs)
    (run,) = glob.glob(os.path.join(out, "mepol", "*"))
    return run


def _csv(path):
    rows = open(path).read().strip().splitlines()
    return rows[0], [r.split(",") for r in rows[1:]]


def test_two_rank_cli_reproduces_one_rank(cuda, tmp_path):
    one = _launch(1, str(tmp_path / "one"))
    two = _launch(2, str(tmp_path / "two"))
    for name, cols in (("MountainCar.csv", (1, 2, 3, 4)),
                       ("MountainCar_off_policy_iter.csv", (0, 1, 2, 3, 4))):
        h1, r1 = _csv(os.path.join(one, name))
        h2, r2 = _csv(os.path.join(two, name))
        assert h1 == h2 and len(r1) == len(r2) and len(r1) > 1
        for a, b in zip(r1, r2):
            for c in cols:
                np.testing.assert_allclose(float(b[c]), float(a[c]), rtol=1e-9, atol=1e-12)
    # rank 0 alone wrote the run directory (one per launch) and the checkpoints
    for e in (0, 2):
        assert os.path.exists(os.path.join(two, f"{e}-policy"))
