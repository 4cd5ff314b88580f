"""Visitation heatmap (get_heatmap, src/algorithms/mepol.py:19-67; Discretizer,
src/envs/discretizer.py:4-26): oracle pinned by the reference's own output, product vs both."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import mepol_oracle as O

CASES = ["mc", "gw", "xy"]


def _disc(z):
    from mepol_amd.envs.discretizer import Discretizer

    tf = (lambda s: [s[0], s[1]]) if bool(z["xy"]) else None
    return Discretizer(z["ranges"].tolist(), z["bins"].tolist(), tf)


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_heatmap(case):
    z = load_golden(f"heatmap_{case}")
    dist, ent = O.heatmap_stats(z["ranges"].tolist(), z["bins"].tolist(), z["visits"][:, :, :2])
    assert np.array_equal(dist, z["dist"])
    assert ent == float(z["entropy"])


@pytest.mark.parametrize("case", CASES)
def test_visitation_stats_match_reference(case):
    z = load_golden(f"heatmap_{case}")
    disc = _disc(z)
    vis = torch.as_tensor(z["visits"].astype(np.float64))
    dist, ent = disc.visitation_stats(vis)
    assert dist.shape == tuple(z["bins"].tolist())
    # counts are exact; only the order of the f64 averaging sums differs (bincount + sum)
    np.testing.assert_allclose(dist.numpy(), z["dist"], rtol=1e-14, atol=0)
    assert abs(float(ent) - float(z["entropy"])) <= 1e-13 * abs(float(z["entropy"]))
    # every visit lands in the bin the reference's np.digitize gives it
    E, T, nf = z["visits"].shape
    rows = z["visits"].reshape(E * T, nf)
    flat = disc.bin_index_torch(vis.reshape(E * T, nf)[:, :2]).numpy()
    ref = np.array([np.ravel_multi_index(disc.discretize(s), disc.bins_sizes) for s in rows])
    assert np.array_equal(flat, ref)


def test_transform_must_select_columns():
    from mepol_amd.envs.discretizer import Discretizer

    d = Discretizer([[-1, 1], [-1, 1]], [4, 4], lambda s: [s[0] * 2, s[1]])
    with pytest.raises(NotImplementedError):
        d.visitation_stats(torch.zeros((1, 3, 3), dtype=torch.float64))
    d = Discretizer([[-1, 1], [-1, 1]], [4, 4], lambda s: [s[2], s[0]])
    vis = torch.as_tensor(np.random.default_rng(0).uniform(-1.2, 1.2, (3, 50, 3)))
    got, h = d.visitation_stats(vis)
    ref, ref_h = O.heatmap_stats([[-1, 1], [-1, 1]], [4, 4], vis.numpy()[:, :, [2, 0]])
    np.testing.assert_allclose(got.numpy(), ref, rtol=1e-14)
    assert abs(float(h) - ref_h) <= 1e-13 * ref_h


def test_heatmap_figure_and_log_rows(tmp_path):
    """The figure follows mepol.py:49-65; the heatmap CSV row and log row are written
    (mepol.py:216-218, 230-233, 247-249)."""
    from mepol_amd.algorithms import mepol as M

    pytest.importorskip("matplotlib")
    dist = np.zeros((4, 3))
    dist[0, 0], dist[1, 2], dist[3, 1] = 0.5, 0.25, 0.25
    fig = M._heatmap_figure(dist, [4, 3], "Blues", None, ("X", "Y"))
    assert fig is not None
    assert M._heatmap_figure(np.array([0.5, 0.5, 0.0]), [3], "Blues", None, ("X", "Y")) is not None

    class Writer:
        def __init__(self):
            self.tags = []

        def add_scalar(self, tag, v, global_step=None):
            self.tags.append(tag)

        def add_figure(self, tag, f, global_step=None):
            self.tags.append(tag)

    w = Writer()
    files = [open(tmp_path / n, "w", encoding="utf-8") for n in ("log.txt", "a.csv", "b.csv")]
    M.log_epoch_statistics(w, files[0], files[1], files[2], 10, -1.0, 1.0, 3, 0.5, 2.0, fig, 4.5,
                           1, 1e-3)
    for f in files:
        f.close()
    assert (tmp_path / "b.csv").read_text() == "10,4.5\n"
    assert "Heatmap" in w.tags and "Discrete entropy" in w.tags
    assert "Heatmap entropy" in (tmp_path / "log.txt").read_text(encoding="utf-8")


def test_cli_specs_build_reference_discretizers():
    from mepol_amd.envs import ErgodicEnv, GridWorldContinuous, MountainCarContinuous
    from mepol_amd.experiments.mepol import exp_specs

    specs = exp_specs()
    mc = specs["MountainCar"]["discretizer_create"](ErgodicEnv(MountainCarContinuous()))
    assert mc.bins_sizes == [12, 11] and mc.feature_ranges == [[-1.2, 0.6], [-0.07, 0.07]]
    gw = specs["GridWorld"]["discretizer_create"](ErgodicEnv(GridWorldContinuous()))
    assert gw.bins_sizes == [20, 20] and gw.feature_ranges == [[-6, 6], [-6, 6]]
    assert specs["Ant"]["discretizer_create"](None).feature_columns(29) == [0, 1]
    assert specs["HandReach"]["discretizer_create"](None) is None


@pytest.mark.gpu
@pytest.mark.parametrize("env_name", ["MountainCar", "GridWorld"])
def test_get_heatmap_on_device(cuda, env_name):
    """get_heatmap's device statistics equal the oracle's over the very states the rollout
    visited (recorded in f64), and the recorded states are the rollout's own."""
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.experiments.mepol import exp_specs
    from mepol_amd.policy import GaussianPolicy

    spec = exp_specs()[env_name]
    env = spec["env_create"]()
    disc = spec["discretizer_create"](env)
    torch.manual_seed(1)
    pol = GaussianPolicy([64, 64], 2, env.action_space.shape[0], spec["log_std_init"]).cuda()
    E, T = 12, 400
    vis = torch.empty((E, T, 2), dtype=torch.float64, device="cuda")
    st, _, _, _ = M.collect_particles_device(env, pol, E, T, None, visited=vis)
    # the f32 particle record is the rounded f64 state
    assert torch.equal(st[:, 1:].double(), vis.float().double())
    dist, ent = disc.visitation_stats(vis)
    ref, ref_h = O.heatmap_stats(disc.feature_ranges, disc.bins_sizes, vis.cpu().numpy())
    np.testing.assert_allclose(dist.cpu().numpy(), ref, rtol=1e-14, atol=0)
    assert abs(float(ent) - ref_h) <= 1e-13 * max(ref_h, 1.0)
    d2, h2, _ = M.get_heatmap(env, pol, disc, E, T, spec["heatmap_cmap"], spec["heatmap_interp"],
                              spec["heatmap_labels"])
    assert d2.shape == tuple(disc.bins_sizes) and abs(d2.sum() - 1.0) < 1e-12
    assert 0.0 <= h2 <= np.log(np.prod(disc.bins_sizes))
