"""Fused policy forward (mepol_policy_forward) vs the three-kernel path (layer_forward + rocBLAS
z2 GEMM + head_forward) at the bench shapes.  PROBE_W = workload (C3 / C4 / C5 / C2)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

SHAPES = {"C3": (200000, 29, 400, 300, 8), "C4": (200000, 47, 400, 300, 17),
          "C5": (500000, 63, 400, 300, 20), "C2": (20000, 2, 300, 300, 2)}
dev = torch.device("cuda")
f64 = dict(dtype=torch.float64, device=dev)


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


for w in os.environ.get("PROBE_W", "C3,C4,C5").split(","):
    N, F, H0, H1, A = SHAPES[w]
    torch.manual_seed(0)
    x = torch.randn(N, F, **f64)
    W1, b1 = torch.randn(H0, F, **f64) * 0.2, torch.randn(H0, **f64) * 0.1
    W2, b2 = torch.randn(H1, H0, **f64) * 0.05, torch.randn(H1, **f64) * 0.1
    Wm, bm = torch.randn(A, H1, **f64) * 0.05, torch.randn(A, **f64)
    ls = torch.full((A,), -0.5, **f64)
    act = torch.randn(N, A, **f64)
    h1, z2 = torch.empty(N, H0, **f64), torch.empty(N, H1, **f64)
    mu, lp = torch.empty(N, A, **f64), torch.empty(N, **f64)

    def three():
        ops.layer_forward(x, W1, b1, out=h1)
        torch.mm(h1, W2.t(), out=z2)
        ops.head_forward(z2, Wm, bm, ls, act, bz=b2, mu_out=mu, logp_out=lp)

    def fused():
        ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, h1, z2, mu, lp)

    fl = 2.0 * N * H0 * H1
    ms3, msf = t(three), t(fused)
    print(f"{w}: three-kernel {ms3 * 1e3:8.1f} us   fused {msf * 1e3:8.1f} us "
          f"({fl / msf / 1e9:.1f} TF/s on the z2 GEMM flops)", flush=True)
