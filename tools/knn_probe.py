"""Time the k-NN at BASELINE C3 size (N=200k, d=29, k=30) and variants; used under rocprofv3."""
import argparse
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=200000)
p.add_argument("--d", type=int, default=29)
p.add_argument("--kp1", type=int, default=31)
p.add_argument("--reps", type=int, default=3)
p.add_argument("--split", type=int, default=0)
p.add_argument("--nq", type=int, default=0, help="queries = the first nq rows (0: all)")
p.add_argument("--grid", action="store_true", help="GridWorld-like data: uniform in [-6, 6]^d")
a = p.parse_args()
from mepol_amd import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn((a.n, a.d), device="cuda", generator=g)
if a.grid:
    X = torch.rand((a.n, a.d), device="cuda", generator=g) * 12 - 6
nq = a.nq or a.n
Q = X[:nq]
print(ops.knn_plan(a.n, nq, a.d, a.kp1, a.split))
D, I, I32T, nfb = ops.knn(X, a.kp1, query=Q, split=a.split, return_fallback=True)
torch.cuda.synchronize()
ts = []
for _ in range(a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.knn(X, a.kp1, query=Q, split=a.split)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
F = 3.0 * a.d * nq * a.n
print(f"knn ms {min(ts):.3f} (all {['%.2f' % t for t in ts]})  algorithmic {F / min(ts) / 1e9:.1f} TFLOP/s  "
      f"fallback {int(nfb.item())}")
