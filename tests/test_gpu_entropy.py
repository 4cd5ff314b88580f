"""GPU parity of importance weights, entropy, KL and the policy gradient step.

Each fixture holds the reference's values over 3 optimizer steps (make_golden.py:gen_entropy).
This build recomputes them with its HIP kernels + PyTorch-ROCm MLP (all f64), through the
drop-in functions, and must agree within 1e-9 relative (the north star asks 1e-5).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, state_dict_from

pytestmark = pytest.mark.gpu

ENTROPY = ["entropy_gw", "entropy_mc", "entropy_ant", "entropy_ant_d29", "entropy_gw300",
           "entropy_dup_inf"]
RTOL = 1e-9


def _policy(sd, ls_init=-0.5):
    from mepol_amd.policy import GaussianPolicy

    hidden = [sd[f"net.{i}.weight"].shape[0] for i in range(0, 100, 2) if f"net.{i}.weight" in sd]
    p = GaussianPolicy(hidden, sd["net.0.weight"].shape[1], sd["mean.weight"].shape[0], ls_init)
    p.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    return p.cuda()


def _inputs(z):
    dev = "cuda"
    st = torch.as_tensor(z["states"], dtype=torch.float64, device=dev)
    ac = torch.as_tensor(z["actions"], dtype=torch.float64, device=dev)
    rl = torch.as_tensor(z["rtl"], dtype=torch.int64, device=dev)
    D = torch.as_tensor(z["D"], dtype=torch.float64, device=dev)
    I = torch.as_tensor(z["I"], dtype=torch.int64, device=dev)
    return st, ac, rl, D, I


def _close(got, ref, rtol=RTOL):
    ref = np.asarray(ref, dtype=np.float64)
    got = np.asarray(got, dtype=np.float64)
    if not np.all(np.isfinite(ref)):
        assert np.array_equal(np.isfinite(got), np.isfinite(ref))
        m = np.isfinite(ref)
        got, ref = got[m], ref[m]
        if ref.size == 0:
            return
    scale = max(np.abs(ref).max(), 1e-300)
    assert np.abs(got - ref).max() <= rtol * scale, (np.abs(got - ref).max(), scale)


@pytest.mark.parametrize("name", ENTROPY)
def test_three_optimizer_steps_match_reference(cuda, name):
    from mepol_amd.algorithms import mepol as M

    z = load_golden(name)
    k, eps, G, B, ns = int(z["k"]), float(z["eps"]), float(z["G"]), float(z["B"]), int(z["ns"])
    st, ac, rl, D, I = _inputs(z)
    nt = st.shape[0]
    beh = _policy(state_dict_from(z, "beh."))
    tgt = _policy(state_dict_from(z, "it0.tgt."))
    lr = float(z["lr"])
    opt = (torch.optim.Adam(tgt.parameters(), lr=lr) if str(z["optimizer"]) == "adam"
           else torch.optim.RMSprop(tgt.parameters(), lr=lr))
    for it in range(3):
        for pname, p in tgt.state_dict().items():
            _close(p.cpu().numpy(), z[f"it{it}.tgt.{pname}"], rtol=1e-8)
        with torch.no_grad():
            w = M.compute_importance_weights(beh, tgt, st, ac, nt, rl)
            H = M.compute_entropy(beh, tgt, st, ac, nt, rl, D, I, k, G, B, ns, eps)
        _close(w.cpu().numpy(), z[f"it{it}.w"])
        _close(H.item(), float(z[f"it{it}.H"]))
        loss, nerr = M.policy_update(opt, beh, tgt, st, ac, nt, rl, D, I, k, G, B, ns, eps)
        assert bool(nerr) == bool(z[f"it{it}.nerr"])
        _close(loss.item(), float(z[f"it{it}.loss"]))
        if not bool(z[f"it{it}.nerr"]):
            for pname, p in tgt.named_parameters():
                _close(p.grad.cpu().numpy(), z[f"it{it}.grad.{pname}"], rtol=1e-8)
        kl, kerr = M.compute_kl(beh, tgt, st, ac, nt, rl, D, I, k, eps)
        assert bool(kerr) == bool(z[f"it{it}.kerr"])
        _close(kl.item(), float(z[f"it{it}.kl"]))
    for pname, p in tgt.state_dict().items():
        _close(p.cpu().numpy(), z[f"final.tgt.{pname}"], rtol=1e-7)


def test_iw_autograd_matches_torch(cuda):
    """compute_importance_weights is differentiable like the reference's torch expression."""
    from mepol_amd.algorithms import mepol as M

    z = load_golden("entropy_ant")
    st, ac, rl, D, I = _inputs(z)
    beh = _policy(state_dict_from(z, "beh."))
    tgt = _policy(state_dict_from(z, "it1.tgt."))
    nt, T = ac.shape[:2]
    coef = torch.randn(nt * T, dtype=torch.float64, device="cuda")
    w = M.compute_importance_weights(beh, tgt, st, ac, nt, rl)
    (coef * w).sum().backward()
    got = {n: p.grad.clone() for n, p in tgt.named_parameters()}
    tgt.zero_grad()
    # plain torch restatement of mepol.py:121-138 on the same device
    lt = tgt.get_log_p(st[:, :T].reshape(nt * T, -1), ac.reshape(nt * T, -1)).reshape(nt, T)
    with torch.no_grad():
        lb = beh.get_log_p(st[:, :T].reshape(nt * T, -1), ac.reshape(nt * T, -1)).reshape(nt, T)
    u = torch.exp(torch.cumsum(lt - lb, dim=1)).reshape(-1)
    wr = u / u.sum()
    assert torch.allclose(w, wr, rtol=1e-12, atol=0)
    (coef * wr).sum().backward()
    for n, p in tgt.named_parameters():
        assert torch.allclose(got[n], p.grad, rtol=1e-9, atol=1e-12 * p.grad.abs().max().item()), n


def test_entropy_deterministic_and_short_circuit(cuda):
    from mepol_amd.algorithms import mepol as M

    z = load_golden("entropy_gw300")
    k, eps, G, B, ns = int(z["k"]), float(z["eps"]), float(z["G"]), float(z["B"]), int(z["ns"])
    st, ac, rl, D, I = _inputs(z)
    beh = _policy(state_dict_from(z, "beh."), -1.5)
    tgt = _policy(state_dict_from(z, "it1.tgt."), -1.5)
    nt = st.shape[0]
    outs = []
    for _ in range(2):
        tgt.zero_grad()
        H = M.compute_entropy(beh, tgt, st, ac, nt, rl, D, I, k, G, B, ns, eps)
        H.backward()
        outs.append((H.item(), [p.grad.clone() for p in tgt.parameters()]))
    assert outs[0][0] == outs[1][0]
    assert all(torch.equal(a, b) for a, b in zip(outs[0][1], outs[1][1]))
    # target is behavioral -> identical to the behavioral-vs-copy value (IW == 1/N)
    beh2 = _policy(state_dict_from(z, "beh."), -1.5)
    with torch.no_grad():
        h_same = M.compute_entropy(beh, beh, st, ac, nt, rl, D, I, k, G, B, ns, eps).item()
        h_copy = M.compute_entropy(beh, beh2, st, ac, nt, rl, D, I, k, G, B, ns, eps).item()
    assert h_same == h_copy
    _close(h_same, float(z["it0.H"]))
