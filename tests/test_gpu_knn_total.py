"""GPU k-NN beyond the f16 screen's shapes: the C ABI answers every (d, k+1 <= N) that the
reference's NearestNeighbors(n_neighbors=k+1) accepts (src/algorithms/mepol.py:190-192, any
--k from src/experiments/mepol.py:25, any state_filter width), bit-exact against the oracle's
exhaustive f64 scan; and inputs whose f32 squared norms overflow are answered, not refused."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mepol_oracle as O

pytestmark = pytest.mark.gpu


def _knn(X, kp1, query=None, **kw):
    from mepol_amd import ops

    Xt = torch.as_tensor(np.ascontiguousarray(X), dtype=torch.float32, device="cuda")
    Qt = None if query is None else torch.as_tensor(np.ascontiguousarray(query),
                                                    dtype=torch.float32, device="cuda")
    D, I, I32T, nfb = ops.knn(Xt, kp1, query=Qt, return_fallback=True, **kw)
    torch.cuda.synchronize()
    return D.cpu().numpy(), I.cpu().numpy(), I32T.cpu().numpy(), int(nfb.item())


# (n, d, k+1): past the screen's k+1 <= 60 / d <= 63, the LDS block-select capacity
# (k+1 = 3500: lists in the global workspace) and k+1 = n
SHAPES = [(3000, 29, 61), (3000, 29, 65), (2500, 12, 101), (2000, 7, 201), (2500, 64, 31),
          (2000, 100, 31), (1500, 100, 101), (700, 300, 9), (400, 5, 400), (4000, 3, 3500)]


@pytest.mark.parametrize("n,d,kp1", SHAPES)
def test_exhaustive_plan_bitexact_vs_oracle(cuda, n, d, kp1):
    from mepol_amd import ops

    assert ops.knn_plan(n, n, d, kp1)["mode"] == "exhaustive"
    X = np.random.default_rng(n + d + kp1).standard_normal((n, d)).astype(np.float32)
    D, I, I32T, nfb = _knn(X, kp1)
    Do, Io = O.knn_exact(X, kp1)
    assert np.array_equal(D, Do) and np.array_equal(I, Io)
    assert np.array_equal(I32T.T, I)
    assert nfb == n  # every query answered by the exhaustive scan


def test_screen_boundary_shapes_keep_screen():
    """The screen still takes the shipped shapes (C3/C4/C5, GridWorld k = 50)."""
    from mepol_amd import ops

    for n, d, kp1 in [(200000, 29, 31), (200000, 47, 31), (500000, 63, 51), (24000, 2, 51),
                      (5000, 63, 60)]:
        assert ops.knn_plan(n, n, d, kp1)["mode"] == "screened", (n, d, kp1)


@pytest.mark.parametrize("kp1", [61, 101])
def test_exhaustive_plan_ties_vs_oracle(cuda, kp1):
    """GridWorld data with exact duplicates (wall rows): ties by the smaller index."""
    z = load_golden("knn_gw_ties")
    D, I, _, _ = _knn(z["X"], kp1)
    Do, Io = O.knn_exact(z["X"], kp1)
    assert np.array_equal(D, Do) and np.array_equal(I, Io)


def test_exhaustive_plan_query_shard(cuda):
    """Multi-rank form (a query shard against all candidates) with an exhaustive plan."""
    X = np.random.default_rng(11).standard_normal((3000, 80)).astype(np.float32)
    D, I, _, _ = _knn(X, 41, query=X[1000:1700])
    Do, Io = O.knn_exact(X, 41, Q=X[1000:1700])
    assert np.array_equal(D, Do) and np.array_equal(I, Io)


def test_exhaustive_plan_rejects_non_finite(cuda):
    from mepol_amd import ops

    X = np.random.default_rng(2).standard_normal((1000, 70)).astype(np.float32)
    X[321, 69] = np.nan
    with pytest.raises(ValueError, match="NaN or infinity"):
        ops.knn(torch.as_tensor(X, device="cuda"), 31)
    *_, chk = ops.knn(torch.as_tensor(X, device="cuda"), 31, defer_check=True)
    with pytest.raises(ValueError, match="NaN or infinity"):
        chk.raise_if_invalid()


def test_more_neighbours_than_samples_raises(cuda):
    from mepol_amd import ops

    X = torch.randn(50, 4, device="cuda")
    with pytest.raises(ValueError, match="n_neighbors"):
        ops.knn(X, 51)


@pytest.mark.parametrize("deferred", [False, True])
def test_overflowing_norms_answered_exactly(cuda, deferred):
    """Rows whose f32 squared norm overflows (|x| ~ 1e20) are valid sklearn input: the f16
    screen cannot scale them, so every query takes the exhaustive f64 scan (same bits)."""
    from mepol_amd import ops

    rng = np.random.default_rng(9)
    X = rng.standard_normal((2000, 29)).astype(np.float32)
    X[5] *= np.float32(1e20)
    X[1234, 3] = np.float32(3e19)
    Xt = torch.as_tensor(X, device="cuda")
    if deferred:
        D, I, _, nfb, chk = ops.knn(Xt, 31, return_fallback=True, defer_check=True)
        chk.raise_if_invalid()
    else:
        D, I, _, nfb = ops.knn(Xt, 31, return_fallback=True)
    Do, Io = O.knn_exact(X, 31)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)
    assert int(nfb.item()) == 2000


@pytest.mark.parametrize("kp1", [101, 700])
def test_knn_exact_entry_any_k(cuda, kp1):
    from mepol_amd import ops

    X = np.random.default_rng(kp1).standard_normal((2500, 17)).astype(np.float32)
    D, I, _ = ops.knn_exact(torch.as_tensor(X, device="cuda"), kp1)
    Do, Io = O.knn_exact(X, kp1)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)


def test_knn_exact_entry_refuses_beyond_lds(cuda):
    from mepol_amd import ops
    from mepol_amd._lib import MepolError

    X = torch.randn(5000, 3, device="cuda")
    with pytest.raises(MepolError, match="mepol_knn takes any"):
        ops.knn_exact(X, 4000)


@pytest.mark.parametrize("k", [64, 100, 200])
def test_collect_particles_and_compute_knn_any_k(cuda, k):
    """The epoch entry point at k = 64 / 100 / 200 on a GridWorld rollout (duplicate-heavy
    d = 2 data): D, I bit-exact against the oracle."""
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.envs import ErgodicEnv, GridWorldContinuous
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(k)
    env = ErgodicEnv(GridWorldContinuous())
    pol = GaussianPolicy([300, 300], 2, 2, -1.5).cuda()
    st, ac, rl, ns, D, I = M.collect_particles_and_compute_knn(env, pol, 8, 500, None, k, 1)
    assert D.shape == (4000, k + 1) and I.shape == (4000, k + 1)
    Do, Io = O.knn_exact(ns.float().cpu().numpy(), k + 1)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)


@pytest.mark.parametrize("d,k", [(64, 30), (100, 30), (100, 100)])
def test_make_particle_batch_any_width(cuda, d, k):
    """The external-rollout entry (MuJoCo-shaped batches) with a state_filter of d = 64 / 100:
    D, I bit-exact against the oracle and the entropy of the batch finite."""
    from mepol_amd.algorithms import mepol as M

    nt, T = 4, 500
    g = torch.Generator(device="cuda").manual_seed(d + k)
    st = torch.randn((nt, T + 1, d), device="cuda", generator=g, dtype=torch.float64)
    ac = torch.randn((nt, T, 3), device="cuda", generator=g, dtype=torch.float64)
    rl = torch.full((nt, 1), T, dtype=torch.int64, device="cuda")
    ns = st[:, 1:].reshape(-1, d).float().contiguous()
    _, _, _, _, D, I = M.make_particle_batch(st, ac, rl, ns, k)
    Do, Io = O.knn_exact(ns.cpu().numpy(), k + 1)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)
