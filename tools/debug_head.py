import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mepol_amd import policy as P
for (nf, hidden, a) in [(2, [300, 300], 2), (2, [300, 300], 1), (29, [400, 300], 8)]:
    torch.manual_seed(0)
    pol = P.GaussianPolicy(hidden, nf, a, -0.7).cuda()
    n = 20000
    s = torch.randn(n, nf, dtype=torch.float64, device="cuda")
    act = 0.5 * torch.randn(n, a, dtype=torch.float64, device="cuda")
    coef = torch.randn(n, dtype=torch.float64, device="cuda")
    lp = pol.get_log_p(s, act)
    (coef * lp).sum().backward()
    g1 = {k: v.grad.clone() for k, v in pol.named_parameters()}
    pol.zero_grad()
    mu = pol.mean(pol.net(s))
    std = torch.exp(pol.log_std) + 1e-7
    ref = torch.sum(-0.5 * (P.LOG_2PI + 2 * pol.log_std + (act - mu) ** 2 / std ** 2), dim=1)
    (coef * ref).sum().backward()
    for k, v in pol.named_parameters():
        err = (g1[k] - v.grad).abs().max().item()
        print(nf, hidden, a, k, f"maxabs {v.grad.abs().max().item():.3e} err {err:.3e}")
    print("ls grads", g1["log_std"].tolist(), pol.log_std.grad.tolist())
