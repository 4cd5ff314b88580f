"""Fused HIP Gaussian head (csrc/head.hip) == the PyTorch GaussianPolicy.get_log_p math."""
import numpy as np
import pytest
import torch

from oracle import mepol_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nf,hidden,a", [(2, [300, 300], 2), (2, [300, 300], 1), (29, [400, 300], 8),
                                         (7, [64, 100], 3), (5, [33], 4), (47, [400, 300], 17),
                                         (63, [400, 300], 20), (5, [33], 12), (7, [64, 100], 32),
                                         (9, [70, 500], 24)])
def test_fused_head_matches_unfused(cuda, nf, hidden, a):
    from mepol_amd import policy as P

    torch.manual_seed(0)
    pol = P.GaussianPolicy(hidden, nf, a, -0.7).cuda()
    n = 20000
    assert n >= P.SPLITK_MIN_ROWS
    s = torch.randn(n, nf, dtype=torch.float64, device="cuda")
    act = 0.5 * torch.randn(n, a, dtype=torch.float64, device="cuda")
    coef = torch.randn(n, dtype=torch.float64, device="cuda")
    assert pol._fused_head_ok(s, act)
    lp = pol.get_log_p(s, act)
    (coef * lp).sum().backward()
    g_fused = {k: v.grad.clone() for k, v in pol.named_parameters()}
    pol.zero_grad()
    mu = pol.mean(pol.net(s))  # plain nn.Module path
    std = torch.exp(pol.log_std) + 1e-7
    ref = torch.sum(-0.5 * (P.LOG_2PI + 2 * pol.log_std + (act - mu) ** 2 / std ** 2), dim=1)
    (coef * ref).sum().backward()
    assert torch.allclose(lp, ref, rtol=1e-12, atol=1e-12)
    for k, v in pol.named_parameters():
        assert torch.allclose(g_fused[k], v.grad, rtol=1e-10, atol=1e-12 * v.grad.abs().max()), k
    with torch.no_grad():
        assert torch.allclose(pol.get_log_p(s, act), ref, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("nf,hidden,a", [(29, [400, 300], 8), (2, [300, 300], 2), (7, [130, 70], 3),
                                         (47, [400, 300], 17), (63, [400, 300], 20),
                                         (11, [96, 260], 32)])
def test_two_layer_fused_path_matches_nn_modules(cuda, nf, hidden, a):
    """The _TwoLayerLogp path (HIP layer 1 + rocBLAS layer 2 + HIP head) == nn.Linear/ReLU."""
    from mepol_amd import policy as P

    torch.manual_seed(1)
    pol = P.GaussianPolicy(hidden, nf, a, -0.3).cuda()
    n = 30000
    s = torch.randn(n, nf, dtype=torch.float64, device="cuda")
    act = 0.5 * torch.randn(n, a, dtype=torch.float64, device="cuda")
    coef = torch.randn(n, dtype=torch.float64, device="cuda")
    lp = pol.get_log_p(s, act)
    assert lp.grad_fn is not None and "TwoLayer" in type(lp.grad_fn).__name__
    (coef * lp).sum().backward()
    got = {k: v.grad.clone() for k, v in pol.named_parameters()}
    pol.zero_grad()
    mu = pol.mean(pol.net(s))
    std = torch.exp(pol.log_std) + 1e-7
    ref = torch.sum(-0.5 * (P.LOG_2PI + 2 * pol.log_std + (act - mu) ** 2 / std ** 2), dim=1)
    (coef * ref).sum().backward()
    assert torch.allclose(lp, ref, rtol=1e-12, atol=1e-12)
    for k, v in pol.named_parameters():
        assert torch.allclose(got[k], v.grad, rtol=1e-10, atol=1e-12 * v.grad.abs().max()), k


def test_predict_matches_forward(cuda):
    """predict (policy.py:64-67): batch-1, no grad, returns out[0] on the CPU; deterministic
    gives the mean of the batched forward."""
    from mepol_amd import policy as P

    torch.manual_seed(3)
    pol = P.GaussianPolicy([300, 300], 2, 2, -1.5).cuda()
    s = [0.25, -1.5]
    a = pol.predict(s, deterministic=True)
    assert a.device.type == "cpu" and a.shape == (2,) and a.dtype == torch.float64
    mu, _ = pol(torch.tensor([s], dtype=torch.float64, device="cuda"), deterministic=True)
    assert torch.equal(a, mu[0].cpu())
    torch.manual_seed(0)
    b = pol.predict(s)
    assert b.shape == (2,) and not torch.equal(a, b)


@pytest.mark.parametrize("n,nf,hidden,a", [(1000, 29, [400, 300], 8), (777, 2, [300, 300], 2),
                                           (513, 47, [400, 300], 17), (300, 63, [400, 300], 20),
                                           (100, 5, [37, 45], 3), (65, 1, [16, 320], 32),
                                           (64, 33, [401, 17], 9), (1, 4, [8, 8], 1)])
def test_policy_forward_kernel_matches_torch(cuda, n, nf, hidden, a):
    """mepol_policy_forward (csrc/policy_fwd.hip) == the nn.Linear / ReLU / Gaussian
    log-density math of src/policy.py:21-51 in torch f64.  Even h0 runs the split form
    (layer1_kernel + z2_head_kernel, including the 300-wide K tail); odd h0 (37, 401) the
    one-kernel form."""
    from mepol_amd import ops
    from mepol_amd import policy as P

    torch.manual_seed(3)
    pol = P.GaussianPolicy(hidden, nf, a, -0.4).cuda()
    s = torch.randn(n, nf, dtype=torch.float64, device="cuda")
    act = 0.5 * torch.randn(n, a, dtype=torch.float64, device="cuda")
    W1, b1 = pol.net[0].weight.detach(), pol.net[0].bias.detach()
    W2, b2 = pol.net[2].weight.detach(), pol.net[2].bias.detach()
    Wm, bm = pol.mean.weight.detach(), pol.mean.bias.detach()
    ls = pol.log_std.detach()
    h1, z2, mu, logp = ops.policy_forward(s, W1, b1, W2, b2, Wm, bm, ls, act)
    h1_ref = torch.relu(s @ W1.t() + b1)
    z2_ref = h1_ref @ W2.t()
    mu_ref = torch.relu(z2_ref + b2) @ Wm.t() + bm
    std = torch.exp(ls) + 1e-7
    lp_ref = torch.sum(-0.5 * (P.LOG_2PI + 2 * ls + (act - mu_ref) ** 2 / std ** 2), dim=1)
    torch.testing.assert_close(h1, h1_ref, rtol=1e-13, atol=1e-13)
    torch.testing.assert_close(z2, z2_ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(mu, mu_ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(logp, lp_ref, rtol=1e-12, atol=1e-11)


@pytest.mark.parametrize("nf,hidden,a", [(29, [400, 300], 8), (47, [400, 300], 17),
                                         (63, [400, 300], 20), (2, [300, 300], 2)])
def test_fused_logp_and_mean_vs_oracle(cuda, nf, hidden, a):
    """A2/A3 parity on the GPU against the oracle (not the build against itself): get_log_p and
    the mean of the fused large-batch path (policy.py:21-51) vs oracle.log_p / mlp_mean, the
    numpy restatement pinned on the reference's policy fixtures (tests/test_oracle_golden.py)."""
    from mepol_amd import policy as P

    torch.manual_seed(11)
    pol = P.GaussianPolicy(hidden, nf, a, -0.6).cuda()
    n = 20000
    rng = np.random.default_rng(4)
    s = torch.as_tensor(rng.standard_normal((n, nf)), device="cuda")
    act = torch.as_tensor(0.5 * rng.standard_normal((n, a)), device="cuda")
    assert pol._fused_head_ok(s, act)
    sd = {k: v.detach().cpu().numpy() for k, v in pol.state_dict().items()}
    with torch.no_grad():
        lp = pol.get_log_p(s, act).cpu().numpy()
        mu, _ = pol(s, deterministic=True)
    ref_lp = O.log_p(sd, s.cpu().numpy(), act.cpu().numpy())
    ref_mu = O.mlp_mean(sd, s.cpu().numpy())
    np.testing.assert_allclose(lp, ref_lp, rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(mu.cpu().numpy(), ref_mu, rtol=1e-11, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("n, o, i", [(200000, 300, 400), (25000, 300, 400), (62500, 300, 400),
                                     (10007, 37, 53), (999, 300, 400), (3, 16, 80),
                                     (20000, 400, 29)])
def test_weight_grad_matches_torch(cuda, n, o, i):
    """csrc/wgrad.hip: dW = dy^T x (the dW2 of the off-policy iteration) against torch's f64 GEMM
    on the same operands (sums in another order: 1e-10 of the largest entry)."""
    from mepol_amd import ops

    g = torch.Generator(device="cuda").manual_seed(n + o + i)
    dy = torch.randn((n, o), dtype=torch.float64, device="cuda", generator=g)
    x = torch.randn((n, i), dtype=torch.float64, device="cuda", generator=g)
    out = ops.weight_grad(dy, x)
    ref = dy.t() @ x
    assert out.shape == (o, i)
    err = (out - ref).abs().max().item()
    assert err <= 1e-10 * max(ref.abs().max().item(), 1.0), err
    # fixed-order sums: the same bits on a second call, with a caller-owned workspace too
    ws = ops.weight_grad_workspace(n, o, i, dy.device)
    assert torch.equal(ops.weight_grad(dy, x, ws=ws), out)


@pytest.mark.parametrize("n,hidden,a", [(25000, 300, 8), (4099, 300, 17), (777, 64, 3)])
def test_head_backward_phases_match_one_call(cuda, n, hidden, a):
    """mepol_head_backward_phase: the row kernel on one stream and the parameter-gradient reduces
    on another (as the off-policy iteration runs them) give the same bits as the one-call form."""
    from mepol_amd import ops

    g = torch.Generator(device="cuda").manual_seed(n)
    f64 = dict(dtype=torch.float64, device="cuda")
    z = torch.randn(n, hidden, generator=g, **f64)
    bz = 0.1 * torch.randn(hidden, generator=g, **f64)
    Wm = 0.05 * torch.randn(a, hidden, generator=g, **f64)
    ls = torch.full((a,), -0.5, **f64)
    act = torch.randn(n, a, generator=g, **f64)
    mu = torch.randn(n, a, generator=g, **f64)
    gl = torch.randn(n, generator=g, **f64)
    ref = ops.head_backward(gl, z, Wm, ls, act, mu, bz=bz, need_dz=True)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    got = ops.head_backward(gl, z, Wm, ls, act, mu, bz=bz, need_dz=True, reduce_stream=side)
    torch.cuda.current_stream().wait_stream(side)
    *got2, finish = ops.head_backward(gl, z, Wm, ls, act, mu, bz=bz, need_dz=True,
                                      defer_reduce=True)
    finish()
    torch.cuda.synchronize()
    for r, t, t2 in zip(ref, got, got2):
        assert torch.equal(r, t) and torch.equal(r, t2)
