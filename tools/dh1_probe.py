"""Fused dh1 GEMM + layer-1 backward (mepol_dh1_layer1_backward) vs torch.mm + layer_backward
at the C3 shapes (N = 200k, 29 -> 400 -> 300), alone and concurrent with the dW2 split-K GEMM
on a second stream (as in the device iteration)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402
from mepol_amd.policy import _weight_grad  # noqa: E402

N, F, H0, H1 = 200000, 29, 400, 300
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)
torch.manual_seed(0)
x = torch.randn(N, F, **f64)
W1, b1 = torch.randn(H0, F, **f64) * 0.3, torch.randn(H0, **f64) * 0.1
W2 = torch.randn(H1, H0, **f64) * 0.1
h1 = torch.relu(x @ W1.t() + b1)
dz2 = torch.randn(N, H1, **f64)
wsl = ops.layer_workspace(N, F, H0, dev)
wsf = ops.dh1_layer1_workspace(N, H0, F, dev)
side = torch.cuda.Stream()


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def unfused():
    dh1 = torch.mm(dz2, W2)
    return ops.layer_backward(dh1, h1, x, ws=wsl)


def fused():
    return ops.dh1_layer1_backward(dz2, W2.t().contiguous(), h1, x, ws=wsf)


def with_dw2(fn):
    def run():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            _weight_grad(dz2, h1)
        fn()
        cur.wait_stream(side)
    return run


print(f"unfused {t(unfused):8.1f} us   fused {t(fused):8.1f} us   dW2 alone "
      f"{t(lambda: _weight_grad(dz2, h1)):8.1f} us", flush=True)
print(f"with dW2 concurrent: unfused {t(with_dw2(unfused)):8.1f} us   fused "
      f"{t(with_dw2(fused)):8.1f} us", flush=True)
