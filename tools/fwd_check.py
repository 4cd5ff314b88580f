"""Per-output errors of ops.policy_forward against torch f64 (h1, z2, mu, logp, mask) over a few
shapes: localises a forward-kernel mismatch to its stage.  Usage: python tools/fwd_check.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402

f64 = dict(dtype=torch.float64, device="cuda")
for n, nf, h0, h1w, a in [(20000, 29, 400, 300, 8), (20000, 29, 400, 300, 2), (20000, 2, 300, 300, 8),
                          (1000, 29, 400, 300, 8), (100, 5, 38, 45, 3), (65, 1, 16, 320, 32)]:
    torch.manual_seed(0)
    x = torch.randn(n, nf, **f64)
    W1, b1 = torch.randn(h0, nf, **f64) * 0.2, torch.randn(h0, **f64) * 0.1
    W2, b2 = torch.randn(h1w, h0, **f64) * 0.05, torch.randn(h1w, **f64) * 0.1
    Wm, bm = torch.randn(a, h1w, **f64) * 0.05, torch.randn(a, **f64)
    ls = torch.full((a,), -0.7, **f64)
    act = 0.5 * torch.randn(n, a, **f64)
    mask = ops.h1_mask_buffer(n, h0, x.device)
    h1, z2, mu, lp = ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, mask_out=mask)
    h1r = torch.relu(x @ W1.t() + b1)
    z2r = h1r @ W2.t()
    mur = torch.relu(z2r + b2) @ Wm.t() + bm
    sd = torch.exp(ls) + 1e-7
    lpr = torch.sum(-0.5 * (1.8378770664093453 + 2 * ls + (act - mur) ** 2 / sd ** 2), dim=1)
    bits = (h1r > 0).to(torch.int64)
    w = torch.arange(16, device="cuda")
    pad = (-h0) % 16
    mr = (torch.nn.functional.pad(bits, (0, pad)).reshape(n, -1, 16) << w).sum(-1)
    mk = (mask.to(torch.int64) & 0xFFFF)

    def e(u, v):
        return float((u - v).abs().max())

    bad = (mu - mur).abs().amax(1) > 1e-9
    rows = bad.nonzero().flatten()[:8].tolist()
    print(f"n={n} nf={nf} h=[{h0},{h1w}] a={a}: h1 {e(h1, h1r):.1e} z2 {e(z2, z2r):.1e} "
          f"mu {e(mu, mur):.1e} logp {e(lp, lpr):.1e} mask_ok {bool((mk == mr).all())} "
          f"bad_mu_rows {int(bad.sum())} first {rows}", flush=True)
    if rows:
        r = rows[0]
        print("   mu", mu[r].tolist(), "\n   ref", mur[r].tolist(), flush=True)
