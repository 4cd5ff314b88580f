"""One launch each of the fused forward, the fused dh1 + layer-1 backward and the dW2 kernel at the C3 shapes
(for PMC passes: rocprofv3 --pmc ... -- python tools/mlp_kernels_once.py)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

N, F, H0, H1, A = 200000, 29, 400, 300, 8
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)
torch.manual_seed(0)
x = torch.randn(N, F, **f64)
W1, b1 = torch.randn(H0, F, **f64) * 0.2, torch.randn(H0, **f64) * 0.1
W2, b2 = torch.randn(H1, H0, **f64) * 0.05, torch.randn(H1, **f64) * 0.1
Wm, bm = torch.randn(A, H1, **f64) * 0.05, torch.randn(A, **f64)
ls = torch.full((A,), -0.5, **f64)
act = torch.randn(N, A, **f64)
h1, z2, mu, lp = ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act)
dz2 = torch.randn(N, H1, **f64)
W2t = W2.t().contiguous()
ws = ops.dh1_layer1_workspace(N, H0, F, dev)
wsg = ops.weight_grad_workspace(N, H1, H0, dev)
for _ in range(2):
    ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, h1, z2, mu, lp)
    ops.dh1_layer1_backward(dz2, W2t, h1, x, ws=ws)
    ops.weight_grad(dz2, h1, ws=wsg)
torch.cuda.synchronize()
print("done")
