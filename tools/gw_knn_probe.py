"""C2S-shaped GridWorld rollout data for the k-NN: runs bench's rollout set-up (random-init
policy, train_supervised, GPU collect_particles), then the k-NN with its fallback count and the
duplicate structure of the states; saves the next states (tools/../gpurun_out/gw_states.npy).
Usage: python tools/gw_knn_probe.py [epochs]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mepol_amd import ops  # noqa: E402
from mepol_amd.algorithms import mepol as M  # noqa: E402
from mepol_amd.envs import ErgodicEnv, GridWorldContinuous  # noqa: E402
from mepol_amd.policy import GaussianPolicy, train_supervised  # noqa: E402

epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda:0")
torch.manual_seed(0)
env = ErgodicEnv(GridWorldContinuous())
pol = GaussianPolicy([300, 300], 2, 2, -1.5).to(dev)
train_supervised(env, pol, 100, 5000)
torch.cuda.manual_seed(1000)
for ep in range(epochs):
    st, ac, rtl, nxt = M.collect_particles_device(env, pol, 20, 1200, None)
    x = nxt.float().contiguous()
    D, I, I32T, nfb = ops.knn(x, 51, return_fallback=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.knn(x, 51)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    xc = x.cpu().numpy()
    u, cnt = np.unique(xc, axis=0, return_counts=True)
    print(f"epoch {ep}: N={len(xc)} fallback={int(nfb.item())} unique rows={len(u)} "
          f"max dup={cnt.max()} rows in dup groups >51: {int(cnt[cnt > 51].sum())} "
          f"k-th dist==0: {int((D[:, 50] == 0).sum().item())} knn ms {min(ts):.3f}", flush=True)
    if ep == 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.save(os.path.join(ROOT, "gpurun_out", "gw_states.npy"), xc)
