"""Time ops.weight_grad (csrc/wgrad.hip) against the rocBLAS split-K bmm + sum it replaced, at
the policy's dW2 shapes (dz2 [n, 300], h1 [n, 400]).  Usage: python tools/wgrad_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def bmm_path(dy, x, sk=32):
    n = dy.shape[0]
    rows = n // sk
    main = rows * sk
    out = torch.bmm(dy[:main].reshape(sk, rows, -1).transpose(1, 2),
                    x[:main].reshape(sk, rows, -1)).sum(0)
    if main < n:
        out.add_(dy[main:].t() @ x[main:])
    return out


for n in (200000, 25000, 62500, 500000):
    dy = torch.randn((n, 300), dtype=torch.float64, device="cuda")
    x = torch.randn((n, 400), dtype=torch.float64, device="cuda")
    ws = ops.weight_grad_workspace(n, 300, 400, dy.device)
    out = torch.empty((300, 400), dtype=torch.float64, device="cuda")
    t_k = timed(lambda: ops.weight_grad(dy, x, out=out, ws=ws))
    t_b = timed(lambda: bmm_path(dy, x))
    fl = 2.0 * n * 300 * 400
    print(f"n={n}: wgrad {t_k * 1e3:.1f} us ({fl / t_k / 1e9:.1f} TF/s)   rocBLAS split-K bmm + sum "
          f"{t_b * 1e3:.1f} us ({fl / t_b / 1e9:.1f} TF/s)")
