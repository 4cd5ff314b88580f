"""Phase breakdown of the multi-workgroup rollout step (diagnostic; tools/variants/rollout_probe.hip).

Runs the PROBE instance of rollout_mlp_mw_kernel on GridWorld with the C2 policy shape
(2 -> [300, 300] -> 2, 20 trajectories x T steps) and prints, per step, the mean span of each
phase over all workgroups (s_memtime cycles -> us with the in-kernel clock), next to the wall
time of the product kernel (mepol_rollout_mlp) on the same inputs."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(n=20, T=1000, h0=300, h1=300, reps=5):
    from mepol_amd import ops

    lib = ctypes.CDLL(os.path.join(ROOT, "tools/variants/librollout_probe.so"))
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    f = lambda *s, sc=1.0: (torch.randn(*s, generator=g, dtype=torch.float64) * sc).to(dev)
    W1, b1 = f(h0, 2, sc=0.5), f(h0, sc=0.1)
    W2 = f(h1, h0, sc=1.0 / h0 ** 0.5)
    W2t, b2 = W2.t().contiguous(), f(h1, sc=0.1)
    Wm, bm = f(2, h1, sc=1.0 / h1 ** 0.5), f(2, sc=0.1)
    log_std = torch.full((2,), -0.5, dtype=torch.float64, device=dev)
    init32 = torch.zeros((n, 2), dtype=torch.float32, device=dev)
    noise = f(T, n, 2)
    np_ = (h1 + 63) // 64
    st = torch.empty((n, T + 1, 2), dtype=torch.float32, device=dev)
    ac = torch.empty((n, T, 2), dtype=torch.float32, device=dev)
    mail = torch.empty(n * T * np_ * 2, dtype=torch.int64, device=dev)
    err = torch.zeros(2, dtype=torch.int32, device=dev)  # [error flag, dispatch ticket]
    probe = torch.zeros((n * np_, 8), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    res = []
    for r in range(reps):
        mail.fill_(-1)
        err.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = lib.probe_rollout_mw_gridworld(
            P(W1), P(b1), h0, P(W2t), P(b2), h1, P(Wm), P(bm), P(log_std), P(init32), P(noise),
            ctypes.c_int64(n), ctypes.c_int64(T), P(st), P(ac), P(mail), P(err), P(probe),
            ctypes.c_void_p(s.cuda_stream))
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0 and int(err[0].item()) == 0, (rc, int(err[0].item()))
        res.append((e0.elapsed_time(e1), probe.cpu().numpy().copy()))
    ms, pr = res[-1]
    cyc = pr[:, :5].sum(1).astype(np.float64)
    clk = cyc / (pr[:, 6] / 100e6)                      # Hz, per workgroup
    ghz = float(np.median(clk)) / 1e9
    names = ["layer1 + barrier", "layer2 chain", "mean partial + publish", "poll wait",
             "combine + env + barrier"]
    print(f"probe kernel: {ms * 1e3 / T:.2f} us/step (wall, events), clock {ghz:.2f} GHz")
    for k, nm in enumerate(names):
        v = pr[:, k] / T / (ghz * 1e3)
        print(f"  {nm:28s} mean {v.mean():6.3f} us  min {v.min():6.3f}  max {v.max():6.3f}")
    print(f"  polls per step: mean {pr[:, 5].mean() / T:.1f}  max {pr[:, 5].max() / T:.1f}")
    # product kernel on the same inputs
    tms = []
    for r in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.rollout_mlp(1, W1, b1, W2, b2, Wm, bm, log_std, init32, noise, st, ac)
        e1.record()
        torch.cuda.synchronize()
        tms.append(e0.elapsed_time(e1))
    print(f"product mepol_rollout_mlp: {min(tms) * 1e3 / T:.2f} us/step (incl. mail memset)")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
