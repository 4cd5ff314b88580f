"""Probe f64 GEMM variants for the C3 layer-2 shapes (N=200k, 400 -> 300)."""
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


N, I, O = 200000, 400, 300
dt = torch.float64
x = torch.randn(N, I, device="cuda", dtype=dt)
g = torch.randn(N, O, device="cuda", dtype=dt)
W = torch.randn(O, I, device="cuda", dtype=dt)
b = torch.randn(O, device="cuda", dtype=dt)
Wt = W.t().contiguous()
xt = x.t().contiguous()
gt = g.t().contiguous()
fl = 2 * N * I * O / 1e9
for lib in ("default", "hipblaslt", "rocblas"):
    try:
        if lib != "default":
            torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e)
        continue
    res = {}
    try:
        res["fwd addmm"] = t(lambda: torch.addmm(b, x, W.t()))
        res["fwd mm(x,Wt_contig)"] = t(lambda: torch.mm(x, Wt))
        res["fwd (W x^T)^T"] = t(lambda: torch.mm(W, xt))
        res["dX g@W"] = t(lambda: torch.mm(g, W))
        res["dX (W^T g^T)^T"] = t(lambda: torch.mm(Wt, gt))
        for S in (16, 32, 64):
            rows = N // S
            res[f"dW bmm{S}"] = t(lambda: torch.bmm(g.reshape(S, rows, O).transpose(1, 2), x.reshape(S, rows, I)).sum(0))
        res["dW gt@x"] = t(lambda: torch.mm(gt, x))
    except Exception as e:
        print(lib, "error", e)
    print(lib, {k: f"{v:.3f}ms/{fl / v:.1f}TF" for k, v in res.items()}, flush=True)
