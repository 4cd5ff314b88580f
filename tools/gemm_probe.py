"""Probe f64 GEMM shapes of the C3 policy MLP on the GPU (weight-grad split-K variants)."""
import time

import torch


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


N = 200000
dev = "cuda"
for dt in (torch.float64, torch.float32):
    for (i, o) in [(29, 400), (400, 300), (300, 8)]:
        x = torch.randn(N, i, device=dev, dtype=dt)
        g = torch.randn(N, o, device=dev, dtype=dt)
        W = torch.randn(o, i, device=dev, dtype=dt)
        fl = 2 * N * i * o
        res = {"fwd": t(lambda: torch.mm(x, W.t())), "dX": t(lambda: torch.mm(g, W)),
               "dW": t(lambda: torch.mm(g.t(), x))}
        for S in (16, 32, 64, 128):
            rows = (N + S - 1) // S
            pad = rows * S - N
            xx = torch.nn.functional.pad(x, (0, 0, 0, pad)).reshape(S, rows, i)
            gg = torch.nn.functional.pad(g, (0, 0, 0, pad)).reshape(S, rows, o)
            res[f"dW_bmm{S}"] = t(lambda: torch.bmm(gg.transpose(1, 2), xx).sum(0))
        print(dt, (i, o), {k: f"{v:.3f}ms/{fl / v / 1e9:.1f}TF" for k, v in res.items()}, flush=True)
