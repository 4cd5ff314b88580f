"""Time the fused head / layer kernels at the C3 shapes (N=200k, 400 -> 300 -> 8)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

N, F, H1, H2, A = 200000, 29, 400, 300, 8
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
f64 = dict(dtype=torch.float64, device=dev)
x = torch.randn(N, F, generator=g, **f64)
W1 = torch.randn(H1, F, generator=g, **f64) * 0.2
b1 = torch.randn(H1, generator=g, **f64) * 0.1
z = torch.randn(N, H2, generator=g, **f64)
bz = torch.randn(H2, generator=g, **f64) * 0.1
Wm = torch.randn(A, H2, generator=g, **f64) * 0.1
bm = torch.randn(A, generator=g, **f64)
ls = torch.full((A,), -0.5, **f64)
act = torch.randn(N, A, generator=g, **f64)
gl = torch.randn(N, generator=g, **f64)
h1 = torch.empty(N, H1, **f64)
dh = torch.randn(N, H1, generator=g, **f64)


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


mu, lp = ops.head_forward(z, Wm, bm, ls, act, bz=bz)
res = {
    "head_fwd": t(lambda: ops.head_forward(z, Wm, bm, ls, act, bz=bz, mu_out=mu, logp_out=lp)),
    "head_bwd": t(lambda: ops.head_backward(gl, z, Wm, ls, act, mu, bz=bz)),
    "head_bwd_nodz": t(lambda: ops.head_backward(gl, z, Wm, ls, act, mu, bz=bz, need_dz=False)),
    "layer_fwd": t(lambda: ops.layer_forward(x, W1, b1, out=h1)),
    "layer_bwd": t(lambda: ops.layer_backward(dh, h1, x)),
}
for k, v in res.items():
    print(f"{k:10s} {v:8.1f} us")
