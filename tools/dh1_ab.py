"""dh1 + layer-1 backward (masked form, as the device iteration calls it) at the C3 shapes,
alone and concurrent with the dW2 kernel on a second stream; checked against torch f64.
MEPOL_DH1_NOLDS=0|1 picks the LDS / no-LDS main loop.  Usage: python tools/dh1_ab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

N, F, H0, H1 = 200000, 29, 400, 300
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)
torch.manual_seed(0)
x = torch.randn(N, F, **f64)
W1, b1 = torch.randn(H0, F, **f64) * 0.3, torch.randn(H0, **f64) * 0.1
W2 = torch.randn(H1, H0, **f64) * 0.1
h1 = torch.relu(x @ W1.t() + b1)
dz2 = torch.randn(N, H1, **f64)
W2t = W2.t().contiguous()
mask = ops.h1_mask_buffer(N, H0, dev)
w = torch.arange(16, device=dev)
bits = (h1 > 0).to(torch.int64).reshape(N, -1, 16)
mask.copy_(((bits << w).sum(-1)).to(torch.int16))
ws = ops.dh1_layer1_workspace(N, H0, F, dev)
wsg = ops.weight_grad_workspace(N, H1, H0, dev)
side = torch.cuda.Stream()
dW, db = ops.dh1_layer1_backward(dz2, W2t, h1, x, ws=ws, mask=mask)
dz1 = (dz2 @ W2) * (h1 > 0)
err = max(float((dW - dz1.t() @ x).abs().max()), float((db - dz1.sum(0)).abs().max()))
print(f"max abs err vs torch: {err:.2e} (|dW| ~ {float(dW.abs().max()):.1e})")


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


def alone():
    ops.dh1_layer1_backward(dz2, W2t, h1, x, ws=ws, mask=mask)


def both():
    cur = torch.cuda.current_stream()
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        ops.weight_grad(dz2, h1, ws=wsg)
    ops.dh1_layer1_backward(dz2, W2t, h1, x, ws=ws, mask=mask)
    cur.wait_stream(side)


print(f"dh1 alone {t(alone):.1f} us, dh1 || dW2 {t(both):.1f} us, "
      f"dW2 alone {t(lambda: ops.weight_grad(dz2, h1, ws=wsg)):.1f} us")
