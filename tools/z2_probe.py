"""z2 = h1 W2^T with no LDS (tools/variants/z2_nt.hip) against torch.mm (rocBLAS) and the fused
policy forward (csrc/policy_fwd.hip), C3 shapes.  Build first: bash tools/variants/build_z2.sh"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mepol_amd import ops  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", "libz2_nt.so"))
lib.z2_nt.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                      ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
NAMES = ["64x80 NS2", "64x64 NS2", "64x64 NS3", "32x80 NS3", "64x80 NS1"]


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


f64 = dict(dtype=torch.float64, device="cuda")
N, F, H0, H1, A = 200000, 29, 400, 300, 8
torch.manual_seed(0)
h1 = torch.randn(N, H0, **f64).relu_()
W2 = torch.randn(H1, H0, **f64) * 0.05
z = torch.empty(N, H1, **f64)
st = torch.cuda.current_stream().cuda_stream
ref = h1 @ W2.t()
fl = 2.0 * N * H0 * H1
print(f"rocBLAS mm: {timed(lambda: torch.mm(h1, W2.t(), out=z)) * 1e3:.1f} us", flush=True)
for v, name in enumerate(NAMES):
    z.zero_()
    rc = lib.z2_nt(v, h1.data_ptr(), N, H0, W2.data_ptr(), H1, z.data_ptr(), st)
    torch.cuda.synchronize()
    err = float((z - ref).abs().max() / ref.abs().max())
    ms = timed(lambda: lib.z2_nt(v, h1.data_ptr(), N, H0, W2.data_ptr(), H1, z.data_ptr(), st))
    print(f"{name}: rc {rc} rel err {err:.2e}  {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF/s", flush=True)

x = torch.randn(N, F, **f64)
W1, b1 = torch.randn(H0, F, **f64) * 0.2, torch.randn(H0, **f64) * 0.1
b2 = torch.randn(H1, **f64) * 0.1
Wm, bm = torch.randn(A, H1, **f64) * 0.05, torch.randn(A, **f64)
ls = torch.full((A,), -0.5, **f64)
act = torch.randn(N, A, **f64)
h1o, z2o = torch.empty(N, H0, **f64), torch.empty(N, H1, **f64)
mu, lp = torch.empty(N, A, **f64), torch.empty(N, **f64)
t_f = timed(lambda: ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, h1o, z2o, mu, lp))
t_l = timed(lambda: ops.layer_forward(x, W1, b1, out=h1o))
t_h = timed(lambda: ops.head_forward(z2o, Wm, bm, ls, act, bz=b2, mu_out=mu, logp_out=lp))
print(f"fused forward {t_f * 1e3:.1f} us; layer_forward {t_l * 1e3:.1f} us; head_forward "
      f"{t_h * 1e3:.1f} us", flush=True)
