"""GPU k-NN parity (calls through the C ABI): reference fixtures + oracle at other sizes."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mepol_oracle as O

pytestmark = pytest.mark.gpu

KNN_TIE_FREE = ["knn_mc_d2", "knn_d7", "knn_ant_d29", "knn_hum_d47", "knn_hr_d63", "knn_d30_k30"]


def _knn(X, kp1, **kw):
    from mepol_amd import ops

    Xt = torch.as_tensor(np.ascontiguousarray(X), dtype=torch.float32, device="cuda")
    D, I, I32T, nfb = ops.knn(Xt, kp1, return_fallback=True, **kw)
    torch.cuda.synchronize()
    return D.cpu().numpy(), I.cpu().numpy(), I32T.cpu().numpy(), int(nfb.item())


@pytest.mark.parametrize("name", KNN_TIE_FREE)
def test_knn_matches_reference_fixture(cuda, name):
    z = load_golden(name)
    D, I, I32T, _ = _knn(z["X"], int(z["kp1"]))
    np.testing.assert_allclose(D, z["D"], rtol=4e-16, atol=0)
    assert np.array_equal(I, z["I"].astype(np.int64))
    assert np.array_equal(I32T.T, I)


@pytest.mark.parametrize("nh", ["auto", "1", "2"])
@pytest.mark.parametrize("name", KNN_TIE_FREE + ["knn_gw_ties", "knn_gw_c2"])
def test_knn_bitexact_vs_oracle(cuda, monkeypatch, name, nh):
    """Same f64 arithmetic and the same (distance, index) tie-break as the oracle: bit-exact,
    with the plan's choice of candidate halves and with each one forced (MEPOL_KNN_NH: f16 hi
    only / hi + lo; GridWorld's d = 2 data forced to hi-only sends most queries to the exhaustive
    path, which must give the same bits)."""
    if nh != "auto":
        monkeypatch.setenv("MEPOL_KNN_NH", nh)
    z = load_golden(name)
    kp1 = int(z["kp1"])
    D, I, _, _ = _knn(z["X"], kp1)
    Do, Io = O.knn_exact(z["X"], kp1)
    assert np.array_equal(D, Do)
    assert np.array_equal(I, Io)


@pytest.mark.parametrize("split", [1, 3, 16])
def test_knn_split_invariance(cuda, split):
    z = load_golden("knn_ant_d29")
    D0, I0, _, _ = _knn(z["X"], 31)
    D1, I1, _, _ = _knn(z["X"], 31, split=split)
    assert np.array_equal(D0, D1) and np.array_equal(I0, I1)


@pytest.mark.parametrize("n,d,kp1", [(1, 3, 1), (7, 1, 7), (33, 5, 33), (1000, 63, 51),
                                     (4097, 29, 31), (3001, 12, 5), (2500, 24, 60)])
def test_knn_edge_shapes(cuda, n, d, kp1):
    X = np.random.default_rng(n + d).standard_normal((n, d)).astype(np.float32)
    D, I, _, _ = _knn(X, kp1)
    Do, Io = O.knn_exact(X, kp1)
    assert np.array_equal(D, Do)
    assert np.array_equal(I, Io)


def test_knn_all_duplicates_uses_exact_path(cuda):
    X = np.zeros((500, 3), np.float32)
    X[250:] = 1.0
    D, I, _, nfb = _knn(X, 5)
    Do, Io = O.knn_exact(X, 5)
    assert nfb > 0
    assert np.array_equal(D, Do) and np.array_equal(I, Io)


def test_knn_query_shard_matches_full(cuda):
    """Multi-rank form: a query shard against all candidates == rows of the full result."""
    from mepol_amd import ops

    X = np.random.default_rng(3).standard_normal((3000, 29)).astype(np.float32)
    Xt = torch.as_tensor(X, device="cuda")
    Df, If, _ = ops.knn(Xt, 31)
    Ds, Is, _ = ops.knn(Xt, 31, query=Xt[1000:2200])
    assert torch.equal(Df[1000:2200], Ds) and torch.equal(If[1000:2200], Is)


def test_knn_exact_path_matches_oracle(cuda):
    from mepol_amd import ops

    z = load_golden("knn_gw_ties")
    Xt = torch.as_tensor(z["X"], device="cuda")
    D, I, _ = ops.knn_exact(Xt, 5)
    Do, Io = O.knn_exact(z["X"], 5)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)


def test_knn_large_properties(cuda):
    """BASELINE-size batch (N=200k, d=29, k=30): properties that need no CPU oracle."""
    from mepol_amd import ops

    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn((200000, 29), device="cuda", generator=g, dtype=torch.float32)
    D, I, I32T, nfb = ops.knn(X, 31, return_fallback=True)
    torch.cuda.synchronize()
    assert bool((D[:, 1:] >= D[:, :-1]).all())                  # rows sorted
    assert bool((I[:, 0] == torch.arange(200000, device="cuda")).all())  # self first (tie-free)
    # recomputed distances agree with the reported ones
    sel = torch.randint(0, 200000, (2000,), device="cuda", generator=g)
    Xd = X.double()
    dd = ((Xd[sel][:, None, :] - Xd[I[sel]]) ** 2).sum(-1).sqrt()
    assert torch.allclose(dd, D[sel], rtol=1e-14, atol=0)
    # a sampled subset checked exhaustively against the exact path
    Dq, Iq, _ = ops.knn_exact(X, 31, query=X[sel[:64]])
    assert torch.equal(Dq, D[sel[:64]]) and torch.equal(Iq, I[sel[:64]])
    assert int(nfb.item()) < 200  # certification almost never needs the exhaustive path


@pytest.mark.parametrize("n,d,kp1", [(200000, 29, 31), (200000, 47, 31), (500000, 63, 51)],
                         ids=["C3", "C4", "C5"])
def test_knn_config_sizes_vs_oracle(cuda, n, d, kp1):
    """BASELINE sizes (C3 Ant d=29 k=30, C4 Humanoid d=47 k=30, C5 HandReach N=500k d=63
    k=50) on one GPU: 512 sampled query rows bit-exact against the CPU oracle's exhaustive
    scan (O.knn_exact_sampled), every row sorted with self first."""
    from mepol_amd import ops

    rng = np.random.default_rng(d)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Xt = torch.as_tensor(X, device="cuda")
    D, I, I32T, nfb = ops.knn(Xt, kp1, return_fallback=True)
    torch.cuda.synchronize()
    assert bool((D[:, 1:] >= D[:, :-1]).all())
    assert bool((I[:, 0] == torch.arange(n, device="cuda")).all())
    assert torch.equal(I32T.t().long(), I)
    sel = np.sort(rng.choice(n, 512, replace=False))
    Do, Io = O.knn_exact_sampled(X, kp1, X[sel])
    assert np.array_equal(D[torch.as_tensor(sel, device="cuda")].cpu().numpy(), Do)
    assert np.array_equal(I[torch.as_tensor(sel, device="cuda")].cpu().numpy(), Io)
    assert int(nfb.item()) < n // 1000


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
@pytest.mark.parametrize("where", ["cand", "query"])
def test_knn_rejects_non_finite(cuda, bad, where):
    """sklearn's NearestNeighbors.fit / kneighbors raise ValueError on NaN / inf
    (mepol.py:190-192); the C ABI returns MEPOL_ERR_BAD_ARG, raised as a ValueError."""
    from mepol_amd import ops

    X = np.random.default_rng(0).standard_normal((2000, 29)).astype(np.float32)
    Q = X[:300].copy()
    (X if where == "cand" else Q)[123, 7] = bad
    with pytest.raises(ValueError, match="NaN or infinity"):
        ops.knn(torch.as_tensor(X, device="cuda"), 31, query=torch.as_tensor(Q, device="cuda"))
    # the library stays usable after the rejection
    X[123, 7] = 0.5
    D, I, _ = ops.knn(torch.as_tensor(X, device="cuda"), 31)
    Do, Io = O.knn_exact(X, 31)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)


@pytest.mark.parametrize("bad", [np.nan, np.inf])
@pytest.mark.parametrize("where", ["cand", "query"])
def test_knn_deferred_check(cuda, bad, where):
    """mepol_knn_deferred: no host synchronisation inside the call; the rejection comes from
    the returned check (same ValueError), and a clean call's result is bit-identical to the
    synchronous entry point's."""
    from mepol_amd import ops

    X = np.random.default_rng(1).standard_normal((3000, 29)).astype(np.float32)
    Q = X[:500].copy()
    Xd, Qd = torch.as_tensor(X, device="cuda"), torch.as_tensor(Q, device="cuda")
    D, I, _, chk = ops.knn(Xd, 31, query=Qd, defer_check=True)
    chk.raise_if_invalid()
    D2, I2, _ = ops.knn(Xd, 31, query=Qd)
    assert torch.equal(D, D2) and torch.equal(I, I2)
    (X if where == "cand" else Q)[77, 3] = bad
    *_, chk = ops.knn(torch.as_tensor(X, device="cuda"), 31, query=torch.as_tensor(Q, device="cuda"),
                      defer_check=True)
    with pytest.raises(ValueError, match="NaN or infinity"):
        chk.raise_if_invalid()


def test_make_particle_batch_rejects_non_finite(cuda):
    """The epoch's k-NN (deferred check) raises sklearn's ValueError before returning."""
    from mepol_amd.algorithms import mepol as M

    X = torch.randn(400, 2, device="cuda")
    X[17, 1] = float("nan")
    st = torch.zeros(4, 101, 2, dtype=torch.float64, device="cuda")
    ac = torch.zeros(4, 100, 1, dtype=torch.float64, device="cuda")
    rl = torch.full((4, 1), 100, dtype=torch.int64, device="cuda")
    with pytest.raises(ValueError, match="NaN or infinity"):
        M.make_particle_batch(st, ac, rl, X, 4)


def test_knn_fallback_heavy_input_matches_oracle(cuda):
    """Many uncertified queries (heavy duplicate clusters with near-ties): the chunked
    exhaustive path (exact_kernel over the whole grid + exact_merge_kernel) answers them, and the
    result is still bit-exact against the oracle."""
    rng = np.random.default_rng(5)
    base = rng.standard_normal((40, 12)).astype(np.float32)
    X = np.repeat(base, 60, axis=0)                      # 2400 rows, 40 clusters of 60 copies
    X[::7] += np.float32(1e-6) * rng.standard_normal((len(X[::7]), 12)).astype(np.float32)
    queued = 0
    for kp1 in (5, 31, 60):
        D, I, _, nfb = _knn(X, kp1)
        Do, Io = O.knn_exact(X, kp1)
        assert np.array_equal(D, Do) and np.array_equal(I, Io), kp1
        queued += nfb
    assert queued > 0


@pytest.mark.parametrize("nq", [1, 3, 40])
def test_knn_exact_chunked_few_queries(cuda, nq):
    """Few queued queries spread over the grid (count < 512 blocks: chunked scan + merge):
    bit-exact against the oracle for a query subset with duplicated candidates."""
    from mepol_amd import ops

    rng = np.random.default_rng(nq)
    X = rng.standard_normal((20000, 7)).astype(np.float32)
    X[5000:5100] = X[0]                                   # a cluster of 101 identical rows
    Q = np.concatenate([X[:nq // 2 + 1], rng.standard_normal((nq - nq // 2 - 1, 7))]).astype(
        np.float32)[:nq]
    Xt = torch.as_tensor(X, device="cuda")
    D, I, _, nfb = ops.knn(Xt, 51, query=torch.as_tensor(Q, device="cuda"), return_fallback=True)
    Do, Io = O.knn_exact(X, 51, Q=Q)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)



def test_knn_seed_invariance(cuda, monkeypatch):
    """The cross-range bound seed changes which candidates the partial lists keep (and so how
    many queries refine certifies), never the certified output: D / I with the seed on and off
    are the same bits, on fallback-heavy duplicate clusters and on Ant-shaped data."""
    rng = np.random.default_rng(7)
    base = rng.standard_normal((40, 12)).astype(np.float32)
    Xdup = np.repeat(base, 100, axis=0)
    Xdup[::5] += np.float32(1e-6) * rng.standard_normal((len(Xdup[::5]), 12)).astype(np.float32)
    Xant = rng.standard_normal((6000, 29)).astype(np.float32)
    for X, kp1 in ((Xdup, 31), (Xant, 31)):
        monkeypatch.setenv("MEPOL_KNN_SEED", "1")
        D1, I1, _, _ = _knn(X, kp1, split=3)
        monkeypatch.setenv("MEPOL_KNN_SEED", "0")
        D0, I0, _, _ = _knn(X, kp1, split=3)
        assert np.array_equal(D1, D0) and np.array_equal(I1, I0)
        Do, Io = O.knn_exact(X, kp1)
        assert np.array_equal(D1, Do) and np.array_equal(I1, Io)
    # probe-seeded plans (one k-step half, >= 4 (k + 1) candidates expected below the probe's
    # bound): the probed (2) and published-only (1) seeds certify the same bits
    Xp = rng.standard_normal((9000, 8)).astype(np.float32)
    Xp[1::7] = Xp[::7][: len(Xp[1::7])]  # exact duplicates: ties at the seed
    Do, Io = O.knn_exact(Xp, 2)
    for mode in ("2", "1"):
        monkeypatch.setenv("MEPOL_KNN_SEED", mode)
        D, I, _, _ = _knn(Xp, 2)
        assert np.array_equal(D, Do) and np.array_equal(I, Io), mode
