"""Do a memory-bound HIP kernel and an MFMA-bound f64 GEMM overlap on two streams?

Times (events) at the C3 shapes: the z2 GEMM alone, layer_forward alone, head_backward alone,
and GEMM || layer_forward / GEMM || head_backward launched on two streams."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

N, F, H1, H2, A = 200000, 29, 400, 300, 8
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)
x = torch.randn(N, F, **f64)
W1 = torch.randn(H1, F, **f64) * 0.1
b1 = torch.randn(H1, **f64)
h1 = torch.randn(N, H1, **f64).relu_()
W2 = torch.randn(H2, H1, **f64) * 0.05
z2 = torch.empty(N, H2, **f64)
zz = torch.randn(N, H2, **f64)
Wm = torch.randn(A, H2, **f64) * 0.05
ls = torch.full((A,), -0.5, **f64)
act = torch.randn(N, A, **f64)
mu = torch.randn(N, A, **f64)
g = torch.randn(N, **f64)
h1b = torch.empty(N, H1, **f64)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
wsh = ops.head_workspace(N, H2, A, dev)


def gemm():
    torch.mm(h1, W2.t(), out=z2)


def layer():
    ops.layer_forward(x, W1, b1, out=h1b)


def headb():
    ops.head_backward(g, zz, Wm, ls, act, mu, bz=None, need_dz=True, ws=wsh)


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def both(f1, f2):
    def run():
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            f1()
        with torch.cuda.stream(s2):
            f2()
        cur.wait_stream(s1)
        cur.wait_stream(s2)
    return run


for name, fn in [("gemm", gemm), ("layer_fwd", layer), ("head_bwd", headb),
                 ("gemm+layer serial", lambda: (gemm(), layer())),
                 ("gemm||layer", both(gemm, layer)),
                 ("gemm+head serial", lambda: (gemm(), headb())),
                 ("gemm||head", both(gemm, headb))]:
    print(f"{name:20s} {t(fn):.3f} ms", flush=True)
