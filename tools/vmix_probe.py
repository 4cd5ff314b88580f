"""Does a VALU (DPP) f64 GEMM overlap an MFMA-bound kernel on another stream?  Times the fused
dh1 + layer-1 backward (MFMA) alone, a 48-GF GEMM alone on the VALU (mepol_gemm_dpp) and on the
MFMA (mepol_gemm_nt), and each GEMM concurrently with the dh1 kernel."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import _lib, ops  # noqa: E402

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
ws = ops.dh1_layer1_workspace(N, H0, F, dev)
A = torch.randn(N, H0, **f64)
B = torch.randn(H1, H0, **f64)
C = torch.empty(N, H1, **f64)
side = torch.cuda.Stream()


# the DPP GEMM experiment lives outside the product library (tools/variants/build_dpp.sh)
_DPP = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants",
                                "libdpp_gemm.so")).mepol_gemm_dpp
_DPP.argtypes = _lib.SIGNATURES["mepol_gemm_nt"]


def dpp(variant):
    def run():
        assert _DPP(_lib.ptr(A), N, H0, H0, _lib.ptr(B), H1, H0, None, 0, _lib.ptr(C), H1,
                    variant, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    return run


def mfma():
    ops.gemm_nt(A, B, out=C, variant=9)


def dh1():
    ops.dh1_layer1_backward(dz2, W2t, h1, x, ws=ws)


def both(g):
    def run():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            g()
        dh1()
        cur.wait_stream(side)
    return run


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


print(f"dh1 alone {t(dh1):8.1f} us", flush=True)
for name, g in (("mfma gemm", mfma), ("dpp gemm v5", dpp(5)), ("dpp gemm v8", dpp(8))):
    print(f"{name}: alone {t(g):8.1f} us   with dh1 concurrent {t(both(g)):8.1f} us", flush=True)
