"""Time ops.policy_forward at the C3 policy shape (N=200k, 29->[400,300]->8, f64) for
rocprofv3 kernel stats (layer1_kernel / z2_head_kernel).  Usage: python tools/l1_probe.py [reps]
(L1_N=rows overrides N, e.g. 25000 for the per-rank share of an 8-GPU run)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
f64 = dict(dtype=torch.float64, device="cuda")
n, nf, h0, h1w, a = int(os.environ.get("L1_N", 200000)), 29, 400, 300, 8
torch.manual_seed(0)
x = torch.randn(n, nf, **f64)
W1, b1 = torch.randn(h0, nf, **f64) * 0.2, torch.randn(h0, **f64) * 0.1
W2, b2 = torch.randn(h1w, h0, **f64) * 0.05, torch.randn(h1w, **f64) * 0.1
Wm, bm = torch.randn(a, h1w, **f64) * 0.05, torch.randn(a, **f64)
ls = torch.full((a,), -0.7, **f64)
act = 0.5 * torch.randn(n, a, **f64)
mask = ops.h1_mask_buffer(n, h0, x.device)
for _ in range(reps):
    ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, mask_out=mask)
torch.cuda.synchronize()
print("done")
