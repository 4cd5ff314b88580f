"""f64 GEMM kernels (csrc/gemm.hip): the MFMA tilings and the DPP-VALU experiment == torch f64."""

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


@pytest.mark.parametrize("n,nf,h0,h1w,a", [(200000, 29, 400, 300, 8), (20000, 2, 300, 300, 2),
                                           (4097, 47, 400, 300, 17), (333, 5, 37, 46, 3),
                                           (1000, 63, 400, 300, 20)])
def test_h1_mask_and_masked_dh1(cuda, n, nf, h0, h1w, a):
    """policy_forward(mask_out=...) writes relu'(h1) as bits (word w of row r, bit b:
    h1[r][16 w + b] > 0) and dh1_layer1_backward(mask=...) gives the same bits as the h1 path."""
    from mepol_amd import ops

    torch.manual_seed(n + h0)
    f64 = dict(dtype=torch.float64, device="cuda")
    x = torch.randn(n, nf, **f64)
    W1, b1 = torch.randn(h0, nf, **f64) * 0.3, torch.randn(h0, **f64) * 0.1
    W2, b2 = torch.randn(h1w, h0, **f64) * 0.1, torch.randn(h1w, **f64) * 0.1
    Wm, bm = torch.randn(a, h1w, **f64) * 0.1, torch.randn(a, **f64)
    ls = torch.full((a,), -0.5, **f64)
    act = torch.randn(n, a, **f64)
    mask = ops.h1_mask_buffer(n, h0, x.device)
    h1, z2, mu, lp = ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act, mask_out=mask)
    h1r, z2r, mur, lpr = ops.policy_forward(x, W1, b1, W2, b2, Wm, bm, ls, act)
    assert torch.equal(h1, h1r) and torch.equal(z2, z2r) and torch.equal(lp, lpr)
    pos = torch.nn.functional.pad(h1 > 0, (0, mask.shape[1] * 16 - h0)).view(n, -1, 16)
    want = (pos.to(torch.int32) << torch.arange(16, device="cuda", dtype=torch.int32)).sum(-1)
    assert torch.equal(mask.to(torch.int32) & 0xFFFF, want)
    dz2 = torch.randn(n, h1w, **f64)
    W2t = W2.t().contiguous()
    dW1, db1 = ops.dh1_layer1_backward(dz2, W2t, h1, x)
    dW1m, db1m = ops.dh1_layer1_backward(dz2, W2t, h1, x, mask=mask)
    assert torch.equal(dW1, dW1m) and torch.equal(db1, db1m)
    if h0 % 2 == 0:  # W2 as stored, transposed on the way into LDS (mepol_dh1_layer1_backward_w2)
        dW1w, db1w = ops.dh1_layer1_backward(dz2, None, h1, x, mask=mask, w2=W2)
        assert torch.equal(dW1, dW1w) and torch.equal(db1, db1w)
