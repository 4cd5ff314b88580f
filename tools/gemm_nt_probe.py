"""Time and check mepol_gemm_nt tilings against torch.mm (rocBLAS/hipBLASLt) at the C3 layer-2
shapes: z2 = h1 W2^T (200000 x 400 -> 300) and dh1 = dz2 W2 (200000 x 300 -> 400)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

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


N = int(os.environ.get("PROBE_N", "200000"))
variants = [int(v) for v in os.environ.get("PROBE_VARIANTS", "0,1,2,3,5").split(",")]
KIND = os.environ.get("PROBE_KIND", "nt")  # nt (MFMA) | dpp (VALU, DPP broadcast)
if KIND == "dpp":
    import ctypes

    from mepol_amd import _lib

    # the DPP GEMM experiment lives outside the product library (tools/variants/build_dpp.sh)
    _fn = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "variants",
                                   "libdpp_gemm.so")).mepol_gemm_dpp
    _fn.argtypes = _lib.SIGNATURES["mepol_gemm_nt"]

    def _dpp(A, B, bias, relu=False, out=None, variant=0):
        n, k = A.shape
        C = out if out is not None else torch.empty((n, B.shape[0]), **f64)
        rc = _fn(_lib.ptr(A), n, k, A.stride(0), _lib.ptr(B), B.shape[0], B.stride(0),
                 _lib.ptr(bias), int(relu), _lib.ptr(C), C.stride(0), variant,
                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
        return C

    ops.gemm_nt = _dpp
torch.manual_seed(0)
for K, M, name in ((400, 300, "fwd z2"), (300, 400, "dh1")):
    A = torch.randn(N, K, **f64)
    B = torch.randn(M, K, **f64)
    bias = torch.randn(M, **f64)
    ref = torch.relu(torch.addmm(bias, A, B.t()))
    fl = 2.0 * N * K * M
    ms = t(lambda: torch.mm(A, B.t()))
    print(f"{name}: torch.mm {ms * 1e3:8.1f} us {fl / ms / 1e9:6.1f} TF/s", flush=True)
    for v in variants:
        C = ops.gemm_nt(A, B, bias, relu=True, variant=v)
        err = (C - ref).abs().max().item() / ref.abs().max().item()
        ms = t(lambda: ops.gemm_nt(A, B, bias, relu=True, out=C, variant=v))
        print(f"{name}: variant {v} {ms * 1e3:8.1f} us {fl / ms / 1e9:6.1f} TF/s  rel err {err:.2e}",
              flush=True)
