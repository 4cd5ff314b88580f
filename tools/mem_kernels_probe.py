"""HBM-bound policy kernels at the C3 shapes (N = 200k, 29 -> [400, 300] -> 8): time (HIP events)
and effective bandwidth (compulsory bytes / time) of layer_forward, layer_backward,
head_forward and head_backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

N, F, H1, H2, A = 200000, 29, 400, 300, int(os.environ.get("PROBE_A", "8"))
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)
torch.manual_seed(0)
x = torch.randn(N, F, **f64)
W1 = torch.randn(H1, F, **f64) * 0.1
b1 = torch.randn(H1, **f64)
h1 = torch.empty(N, H1, **f64)
dh1 = torch.randn(N, H1, **f64)
z2 = torch.randn(N, H2, **f64)
b2 = torch.randn(H2, **f64) * 0.1
Wm = torch.randn(A, H2, **f64) * 0.05
bm = torch.randn(A, **f64)
ls = torch.full((A,), -0.5, **f64)
act = torch.randn(N, A, **f64)
mu = torch.empty(N, A, **f64)
logp = torch.empty(N, **f64)
g = torch.randn(N, **f64)
wsh = ops.head_workspace(N, H2, A, dev)
wsl = ops.layer_workspace(N, F, H1, dev)
ops.layer_forward(x, W1, b1, out=h1)


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


rows = [
    ("layer_forward", lambda: ops.layer_forward(x, W1, b1, out=h1), 8 * N * (F + H1)),
    ("layer_backward", lambda: ops.layer_backward(dh1, h1, x, ws=wsl), 8 * N * (F + 2 * H1)),
    ("head_forward", lambda: ops.head_forward(z2, Wm, bm, ls, act, bz=b2, mu_out=mu,
                                              logp_out=logp), 8 * N * (H2 + 2 * A + 1)),
    ("head_backward", lambda: ops.head_backward(g, z2, Wm, ls, act, mu, bz=b2, need_dz=True,
                                                ws=wsh), 8 * N * (2 * H2 + 2 * A + 1)),
]
for name, fn, nbytes in rows:
    ms = t(fn)
    print(f"{name:16s} {ms * 1e3:8.1f} us  {nbytes / ms / 1e6:7.0f} GB/s", flush=True)
