"""f64 GEMM kernels (csrc/gemm.hip): the MFMA tilings and the DPP-VALU experiment == torch f64."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(1000, 400, 300), (333, 30, 50), (64, 16, 16), (1, 2, 7), (2049, 302, 401)]


@pytest.mark.parametrize("n,k,m", SHAPES)
@pytest.mark.parametrize("variant", [0, 1, 6, 9])
def test_gemm_nt_matches_torch(cuda, n, k, m, variant):
    from mepol_amd import ops

    torch.manual_seed(n + k + m)
    A = torch.randn(n, k, dtype=torch.float64, device="cuda")
    B = torch.randn(m, k, dtype=torch.float64, device="cuda")
    bias = torch.randn(m, dtype=torch.float64, device="cuda")
    ref = torch.relu(torch.addmm(bias, A, B.t()))
    out = ops.gemm_nt(A, B, bias, relu=True, variant=variant)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(ops.gemm_nt(A, B, variant=variant), A @ B.t(), rtol=1e-12,
                               atol=1e-12)


def test_gemm_nt_rejects_odd_k(cuda):
    from mepol_amd import _lib, ops

    A = torch.randn(10, 3, dtype=torch.float64, device="cuda")
    with pytest.raises(_lib.MepolInputError):
        ops.gemm_nt(A, A)


@pytest.mark.parametrize("n,nf,h0,h1w", [(200, 29, 400, 300), (1000, 2, 300, 300),
                                         (513, 47, 400, 300), (300, 63, 400, 300),
                                         (77, 5, 37, 46), (4097, 15, 96, 80), (1, 16, 16, 2)])
def test_dh1_layer1_backward_matches_torch(cuda, n, nf, h0, h1w):
    """Fused dh1 GEMM + layer-1 backward == torch: dh1 = dz2 W2, dz1 = dh1 * (h1 > 0),
    dW1 = dz1^T x, db1 = sum dz1 (nn.Linear/ReLU backward of src/policy.py:21-26)."""
    from mepol_amd import ops

    torch.manual_seed(n + nf)
    x = torch.randn(n, nf, dtype=torch.float64, device="cuda")
    W1 = torch.randn(h0, nf, dtype=torch.float64, device="cuda") * 0.3
    b1 = torch.randn(h0, dtype=torch.float64, device="cuda") * 0.1
    W2 = torch.randn(h1w, h0, dtype=torch.float64, device="cuda") * 0.1
    h1 = torch.relu(x @ W1.t() + b1)
    dz2 = torch.randn(n, h1w, dtype=torch.float64, device="cuda")
    dW1, db1 = ops.dh1_layer1_backward(dz2, W2.t().contiguous(), h1, x)
    dz1 = (dz2 @ W2) * (h1 > 0)
    torch.testing.assert_close(dW1, dz1.t() @ x, rtol=1e-11, atol=1e-11)
    torch.testing.assert_close(db1, dz1.sum(0), rtol=1e-11, atol=1e-11)


@pytest.mark.parametrize("n,nf,h0,h1w,a", [(200000, 29, 400, 300, 8), (5000, 29, 400, 300, 8),
                                           (4097, 2, 300, 300, 2), (777, 7, 96, 80, 1),
                                           (33, 5, 64, 46, 3)])
def test_fused_head_backward_matches_round3_path_and_torch(cuda, n, nf, h0, h1w, a):
    """The head backward with dz2 formed on chip (csrc/head_grad.hip + the formed dh1 kernel)
    == head_backward (dz2 written) + dz2^T h1 + dh1_layer1_backward, and == torch autograd of
    get_log_p (src/policy.py:43-51) through relu(z2 + b2) and relu(x W1^T + b1)."""
    from mepol_amd import ops

    torch.manual_seed(n + a)
    f64 = dict(dtype=torch.float64, device="cuda")
    x = torch.randn(n, nf, **f64)
    W1 = torch.randn(h0, nf, **f64) * 0.3
    b1 = torch.randn(h0, **f64) * 0.1
    W2 = torch.randn(h1w, h0, **f64) * 0.1
    b2 = torch.randn(h1w, **f64) * 0.1
    Wm = torch.randn(a, h1w, **f64) * 0.1
    bm = torch.randn(a, **f64) * 0.1
    ls = torch.randn(a, **f64) * 0.2 - 0.5
    act = torch.randn(n, a, **f64) * 0.5
    grad = torch.randn(n, **f64) * 1e-3
    h1 = torch.relu(x @ W1.t() + b1)
    z2 = h1 @ W2.t()
    mu = torch.relu(z2 + b2) @ Wm.t() + bm
    W2t = W2.t().contiguous()
    # round 3 path
    dz2, dWm_r, dbm_r, dls_r, db2_r = ops.head_backward(grad, z2, Wm, ls, act, mu, bz=b2)
    dW2_r = dz2.t() @ h1
    dW1_r, db1_r = ops.dh1_layer1_backward(dz2, W2t, h1, x)
    # fused path
    ws = ops.head_grad_workspace(n, h1w, h0, a, x.device)
    ops.head_coef(grad, act, mu, ls, ws)
    dW2, db2, dWm, dbm, dls = ops.head_dw2(z2, b2, Wm, h1, ws)
    dW1, db1 = ops.dh1_layer1_backward_formed(z2, b2, Wm, ws, W2, h1, x)
    # the formed dz2 is head_bwd's dz2 bit for bit, so dh1 / dW1 only differ by nothing
    assert torch.equal(dW1, dW1_r) and torch.equal(db1, db1_r)
    for got, ref in ((dW2, dW2_r), (db2, db2_r), (dWm, dWm_r), (dbm, dbm_r), (dls, dls_r)):
        torch.testing.assert_close(got, ref, rtol=1e-11, atol=1e-13 * ref.abs().max().item())
    if n <= 5000:  # torch autograd of the reference head (float64)
        P = [t.clone().requires_grad_(True) for t in (W2, b2, Wm, bm, ls)]
        W2_, b2_, Wm_, bm_, ls_ = P
        mu_ = torch.relu(h1 @ W2_.t() + b2_) @ Wm_.t() + bm_
        sd = torch.exp(ls_) + 1e-7
        lp = (-0.5 * (np.log(2 * np.pi) + 2 * ls_ + (act - mu_) ** 2 / sd ** 2)).sum(1)
        (lp * grad).sum().backward()
        for got, p in zip((dW2, db2, dWm, dbm, dls), P):
            torch.testing.assert_close(got, p.grad, rtol=1e-10, atol=1e-12 * p.grad.abs().max().item())
