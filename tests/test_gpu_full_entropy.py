"""The epoch-0 full-entropy path and the deterministic single-state predict, against the oracle.

mepol() logs a "full entropy" every epoch from a separate batch: num_traj x full_entropy_traj_scale
trajectories, the k-NN at full_entropy_k, B recomputed for that k, and the behavioural policy as
its own target (mepol.py:337-354), so the importance weights are uniform.  Here that batch runs
through the drop-in functions (GPU rollout, HIP k-NN, HIP entropy) and is checked against
O.knn_exact + O.importance_weights + O.entropy over the same particles.

predict(s, deterministic=True) is the batch-1 action of policy.py:64-67; checked against
the reference's own means and O.mlp_mean on the fixture states (tests/golden/policy_*.npz)."""
import numpy as np
import pytest
import scipy.special
import torch

from conftest import load_golden, state_dict_from
from oracle import mepol_oracle as O

pytestmark = pytest.mark.gpu


# GridWorld rollouts revisit states exactly (blocked moves at the walls), so with eps = 0 a
# duplicate-heavy batch gives d_k = 0 and H = -inf, in the reference as here; eps = 1e-15 (the
# experiments' value for MountainCar, experiments/mepol.py) keeps it finite.
@pytest.mark.parametrize("num_traj,scale,traj_len,fe_k,eps", [(4, 2, 400, 4, 1e-15),
                                                              (2, 5, 250, 4, 1e-15),
                                                              (3, 2, 300, 7, 1e-15),
                                                              (4, 2, 400, 4, 0.0)])
def test_full_entropy_batch_matches_oracle(cuda, num_traj, scale, traj_len, fe_k, eps):
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.envs import ErgodicEnv, GridWorldContinuous
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(num_traj * 100 + scale)
    env = ErgodicEnv(GridWorldContinuous())
    pol = GaussianPolicy([300, 300], 2, 2, -1.5).cuda()
    nt = num_traj * scale
    st, ac, rl, ns_, D, I = M.collect_particles_and_compute_knn(env, pol, nt, traj_len, None,
                                                                fe_k, 1)
    assert st.shape == (nt, traj_len + 1, 2) and D.shape == (nt * traj_len, fe_k + 1)
    ns = env.num_features
    G = scipy.special.gamma(ns / 2 + 1)
    full_B = np.log(fe_k) - scipy.special.digamma(fe_k)
    with torch.no_grad():
        H = M.compute_entropy(pol, pol, st, ac, nt, rl, D, I, fe_k, G, full_B, ns, eps)
    assert H.device.type == "cpu" and H.dtype == torch.float64 and H.dim() == 0

    # oracle over the same particles
    X = ns_.cpu().numpy()
    Do, Io = O.knn_exact(X.astype(np.float32), fe_k + 1)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)
    sd = {k: v.detach().cpu().numpy() for k, v in pol.state_dict().items()}
    S = st.cpu().numpy()[:, :-1]
    A = ac.cpu().numpy()
    lp = O.log_p(sd, S.reshape(-1, 2), A.reshape(-1, 2)).reshape(nt, traj_len)
    w = O.importance_weights(lp, lp, [traj_len] * nt)
    np.testing.assert_array_equal(w, np.full(nt * traj_len, 1.0 / (nt * traj_len)))
    H_ref = O.entropy(w, Do, Io, fe_k, G, full_B, ns, eps)
    if not np.isfinite(H_ref):
        assert eps == 0.0 and float(H) == H_ref  # -inf on both sides
    else:
        np.testing.assert_allclose(float(H), H_ref, rtol=1e-9)


@pytest.mark.parametrize("name", ["policy_gw", "policy_ant", "policy_pretrained_gw"])
def test_predict_deterministic_matches_oracle(cuda, name):
    from mepol_amd.policy import GaussianPolicy

    z = load_golden(name)
    sd = state_dict_from(z, "sd.")
    hidden = [sd[f"net.{i}.weight"].shape[0] for i in range(0, 100, 2) if f"net.{i}.weight" in sd]
    nf, na = sd["net.0.weight"].shape[1], sd["mean.weight"].shape[0]
    p = GaussianPolicy(hidden, nf, na, -0.5)
    p.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()})
    p = p.cuda()
    # the fixture's rows: the reference's own deterministic means (forward(x, True)) and the
    # oracle's restatement
    for s, ref in zip(z["x"][:8], z["mean"][:8]):
        a = p.predict(s, deterministic=True)
        assert a.device.type == "cpu" and a.dtype == torch.float64 and a.shape == (na,)
        np.testing.assert_allclose(a.numpy(), ref, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(a.numpy(), O.mlp_mean(sd, s[None])[0], rtol=1e-12,
                                   atol=1e-14)
    # the stochastic form draws mean + N(0, 1) exp(log_std): same shape, different value
    a1 = p.predict(s, deterministic=False)
    assert a1.shape == (na,) and not torch.equal(a1, p.predict(s, deterministic=True))
