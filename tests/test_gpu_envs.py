"""GPU env steppers and the fused rollout step vs the reference steps / oracle rollout."""
import numpy as np
import pytest
import torch

from conftest import load_golden, state_dict_from
from oracle import mepol_oracle as O

pytestmark = pytest.mark.gpu


def test_gridworld_step_bitexact(cuda):
    from mepol_amd import ops

    z = load_golden("env_gw")
    s = torch.as_tensor(z["S"], device="cuda").contiguous()
    a = torch.as_tensor(z["A"], dtype=torch.float64, device="cuda")
    ops.step_gridworld(s, a)
    assert np.array_equal(s.cpu().numpy(), z["NS"])


def test_mountaincar_step(cuda):
    from mepol_amd import ops

    z = load_golden("env_mc")
    s = torch.as_tensor(z["S"], dtype=torch.float64, device="cuda").contiguous()
    a = torch.as_tensor(z["A"], dtype=torch.float64, device="cuda")
    ops.step_mountaincar(s, a)
    got = s.cpu().numpy()
    # cos() may differ from glibc in the last ulp; everything else is the same IEEE sequence
    np.testing.assert_allclose(got, z["NS"], rtol=0, atol=1e-15)
    assert (got == z["NS"]).mean() > 0.95


@pytest.mark.parametrize("env", ["mountaincar", "gridworld"])
def test_rollout_with_injected_noise_matches_oracle(cuda, env):
    from mepol_amd import ops
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(5)
    a_dim = 1 if env == "mountaincar" else 2
    pol = GaussianPolicy([32, 32], 2, a_dim, -0.5 if env == "mountaincar" else -1.5).cuda()
    nt, T = 16, 200
    rng = np.random.default_rng(0)
    if env == "mountaincar":
        init = np.stack([rng.uniform(-0.6, -0.4, nt), np.zeros(nt)], 1)
    else:
        init = rng.uniform(-6, -4, (nt, 2)).astype(np.float32)
    noise = rng.standard_normal((T, nt, a_dim))
    sd = {k: v.detach().cpu().numpy() for k, v in pol.state_dict().items()}
    S_ref, A_ref = O.rollout(env, sd, sd["log_std"], init, noise, T)

    dev = "cuda"
    states = torch.zeros((nt, T + 1, 2), dtype=torch.float32, device=dev)
    actions = torch.zeros((nt, T, a_dim), dtype=torch.float32, device=dev)
    env_id = 0 if env == "mountaincar" else 1
    init_t = torch.as_tensor(init, device=dev)
    env64 = init_t.clone().double() if env_id == 0 else None
    env32 = init_t.clone().float() if env_id == 1 else None
    pin = init_t.double().contiguous()
    states[:, 0] = init_t.float()
    nz = torch.as_tensor(noise, dtype=torch.float64, device=dev)
    with torch.no_grad():
        for t in range(T):
            mean = pol.mean_action(pin).contiguous()
            ops.rollout_step(env_id, env64, env32, mean, nz[t].contiguous(), pol.log_std.detach(),
                             t, T, states, actions, pin)
    S = states.cpu().numpy()
    A = actions.cpu().numpy()
    # The MLP runs on rocBLAS (different summation order than numpy): actions agree to ~1e-15
    # and the f32-recorded trajectories agree to f32 rounding unless a wall/clip boundary is
    # crossed within that rounding (rare); require nearly every recorded value to match.
    assert np.abs(A - A_ref).max() < 1e-5
    frac_exact = (S == S_ref).mean()
    assert frac_exact > 0.99, frac_exact
    assert np.abs(S - S_ref).max() < 1e-3


def test_collect_particles_contract(cuda):
    """collect_particles_and_compute_knn returns the reference's shapes/dtypes (mepol.py:195-202)."""
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.envs import ErgodicEnv, GridWorldContinuous
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(0)
    env = ErgodicEnv(GridWorldContinuous())
    pol = GaussianPolicy([300, 300], 2, 2, -1.5).cuda()
    st, ac, rl, ns, D, I = M.collect_particles_and_compute_knn(env, pol, 20, 1000, None, 4, 1)
    assert st.shape == (20, 1001, 2) and st.dtype == torch.float64
    assert ac.shape == (20, 1000, 2) and ac.dtype == torch.float64
    assert rl.shape == (20, 1) and rl.dtype == torch.int64 and bool((rl == 1000).all())
    assert ns.shape == (20000, 2) and ns.dtype == torch.float64
    assert D.shape == (20000, 5) and D.dtype == torch.float64
    assert I.shape == (20000, 5) and I.dtype == torch.int64
    # states stay inside the grid and off the walls; next_states are states[:, 1:]
    assert bool((st.abs() < 6).all())
    assert torch.equal(ns, st[:, 1:].reshape(-1, 2))
    Do, Io = O.knn_exact(ns.float().cpu().numpy(), 5)
    assert np.array_equal(D.cpu().numpy(), Do) and np.array_equal(I.cpu().numpy(), Io)


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("env_name", ["mountaincar", "gridworld"])
def test_rollout_graph_and_shards_match_eager(cuda, monkeypatch, env_name, fused):
    """The graph-replayed rollout == the eager per-step loop (bitwise), and the shards of a
    2- and 4-way trajectory split concatenate to the one-rank rollout (noise and initial states
    are drawn for all trajectories up front).  fused = 1: the one-launch rollout kernel serves
    both settings (no graph is captured)."""
    monkeypatch.setenv("MEPOL_ROLLOUT_FUSED", fused)
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.envs import ErgodicEnv, GridWorldContinuous, MountainCarContinuous
    from mepol_amd.policy import GaussianPolicy

    base = MountainCarContinuous() if env_name == "mountaincar" else GridWorldContinuous()
    env = ErgodicEnv(base)
    a = env.action_space.shape[0]
    torch.manual_seed(0)
    pol = GaussianPolicy([300, 300], 2, a, -1.0).cuda()

    def roll(graph, shard=None, seed=7):
        monkeypatch.setenv("MEPOL_ROLLOUT_GRAPH", "1" if graph else "0")
        g = torch.Generator(device="cuda").manual_seed(seed)
        return M.collect_particles_device(env, pol, 8, 300, None, generator=g, shard=shard)

    eager = roll(False)
    for rep in range(2):  # capture, then replay of the cached graph
        graph = roll(True)
        for x, y in zip(eager, graph):
            assert torch.equal(x, y)
    assert len(M._ROLLOUT_GRAPHS.get(pol, {})) == (1 if fused == "0" else 0)
    for world in (2, 4):
        parts = [roll(True, shard=(r, world)) for r in range(world)]
        assert torch.equal(torch.cat([p[0] for p in parts]), eager[0])
        assert torch.equal(torch.cat([p[1] for p in parts]), eager[1])
        assert torch.equal(torch.cat([p[3] for p in parts]), eager[3])
    # the parameters are read in place at replay: a changed policy changes the rollout
    with torch.no_grad():
        pol.mean.bias.add_(0.05)
    eager2 = roll(False)
    graph2 = roll(True)
    assert torch.equal(eager2[0], graph2[0]) and not torch.equal(eager2[0], eager[0])


@pytest.mark.parametrize("env", ["mountaincar", "gridworld"])
@pytest.mark.parametrize("kl", ["0", "37", "300"])
def test_rollout_mlp_kernel_matches_oracle(cuda, monkeypatch, env, kl):
    """The one-launch rollout, one workgroup per trajectory (mepol_rollout_mlp: policy MLP +
    noise + env step for all T steps) == the oracle's per-step rollout with the same injected
    noise to the rounding of the MLP's summation order, and == the k-ordered oracle (4 chunks)
    bit for bit; how many W2 rows sit in LDS rather than stream from L2 (MEPOL_ROLLOUT_KL,
    37 = a chunk boundary inside the LDS rows) does not change the result."""
    from mepol_amd import ops
    from mepol_amd.policy import GaussianPolicy

    monkeypatch.setenv("MEPOL_ROLLOUT_KL", kl)
    monkeypatch.setenv("MEPOL_ROLLOUT_MW", "0")
    torch.manual_seed(5)
    a_dim = 1 if env == "mountaincar" else 2
    pol = GaussianPolicy([300, 300], 2, a_dim, -0.5 if env == "mountaincar" else -1.5).cuda()
    nt, T = 16, 200
    rng = np.random.default_rng(0)
    if env == "mountaincar":
        init = np.stack([rng.uniform(-0.6, -0.4, nt), np.zeros(nt)], 1)
    else:
        init = rng.uniform(-6, -4, (nt, 2)).astype(np.float32)
    noise = rng.standard_normal((T, nt, a_dim))
    sd = {k: v.detach().cpu().numpy() for k, v in pol.state_dict().items()}
    S_ref, A_ref = O.rollout(env, sd, sd["log_std"], init, noise, T)
    std_dev = torch.exp(pol.log_std.detach()).cpu().numpy()
    S_ko, A_ko = O.rollout_kordered(env, sd, std_dev, init, noise, T, 4)
    dev = "cuda"
    states = torch.zeros((nt, T + 1, 2), dtype=torch.float32, device=dev)
    actions = torch.zeros((nt, T, a_dim), dtype=torch.float32, device=dev)
    visited = torch.zeros((nt, T, 2), dtype=torch.float64, device=dev)
    l1, l2 = pol.net[0], pol.net[2]
    ops.rollout_mlp(0 if env == "mountaincar" else 1, l1.weight.detach(), l1.bias.detach(),
                    l2.weight.detach(), l2.bias.detach(), pol.mean.weight.detach(),
                    pol.mean.bias.detach(), pol.log_std.detach(), torch.as_tensor(init, device=dev),
                    torch.as_tensor(noise, dtype=torch.float64, device=dev), states, actions,
                    visited)
    S, A = states.cpu().numpy(), actions.cpu().numpy()
    assert np.abs(A - A_ref).max() < 1e-5
    assert (S == S_ref).mean() > 0.99
    assert np.abs(S - S_ref).max() < 1e-3
    assert np.array_equal(visited.cpu().numpy().astype(np.float32), S[:, 1:])
    if env == "gridworld":
        assert np.array_equal(A, A_ko) and np.array_equal(S, S_ko)
    else:
        np.testing.assert_allclose(A, A_ko, rtol=0, atol=1e-12)


def _rollout_inputs(env, hidden, nt, T, seed):
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(seed)
    a_dim = 1 if env == "mountaincar" else 2
    pol = GaussianPolicy(hidden, 2, a_dim, -0.5 if env == "mountaincar" else -1.5).cuda()
    rng = np.random.default_rng(seed)
    if env == "mountaincar":
        init = np.stack([rng.uniform(-0.6, -0.4, nt), np.zeros(nt)], 1)
    else:
        init = rng.uniform(-6, -4, (nt, 2)).astype(np.float32)
    noise = rng.standard_normal((T, nt, a_dim))
    return pol, init, noise


def _rollout_run(env, pol, init, noise):
    from mepol_amd import ops

    T, nt, a_dim = noise.shape
    states = torch.zeros((nt, T + 1, 2), dtype=torch.float32, device="cuda")
    actions = torch.zeros((nt, T, a_dim), dtype=torch.float32, device="cuda")
    l1, l2 = pol.net[0], pol.net[2]
    ops.rollout_mlp(0 if env == "mountaincar" else 1, l1.weight.detach(), l1.bias.detach(),
                    l2.weight.detach(), l2.bias.detach(), pol.mean.weight.detach(),
                    pol.mean.bias.detach(), pol.log_std.detach(),
                    torch.as_tensor(init, device="cuda"),
                    torch.as_tensor(noise, dtype=torch.float64, device="cuda"), states, actions)
    return states, actions


@pytest.mark.parametrize("env", ["mountaincar", "gridworld"])
@pytest.mark.parametrize("hidden", [[300, 300], [64, 48], [400, 300], [2, 130]])
def test_rollout_forms_bit_identical(cuda, monkeypatch, env, hidden):
    """Both forms of mepol_rollout_mlp sum layer 2 in the same 4-chunk order: several
    workgroups per trajectory (MEPOL_ROLLOUT_MW=1) and one (=0) give the same bits, so the host
    may pick either per call (a rank's shard and the one-rank batch can take different forms)."""
    from mepol_amd import ops

    pol, init, noise = _rollout_inputs(env, hidden, 24, 50, 9)
    monkeypatch.setenv("MEPOL_ROLLOUT_MW", "1")
    plan = ops.rollout_mlp_plan(24, hidden[0], hidden[1], noise.shape[2])
    assert plan["k_chunks"] == 4
    assert plan["workgroups_per_traj"] == (1 if hidden[0] > 306 else (hidden[1] + 63) // 64)
    s1, a1 = _rollout_run(env, pol, init, noise)
    monkeypatch.setenv("MEPOL_ROLLOUT_MW", "0")
    assert ops.rollout_mlp_plan(24, hidden[0], hidden[1], noise.shape[2])["workgroups_per_traj"] == 1
    s0, a0 = _rollout_run(env, pol, init, noise)
    assert torch.equal(a1, a0) and torch.equal(s1, s0)


def test_rollout_error_word_reset(cuda, monkeypatch):
    """the error word of a reused rollout workspace is zeroed by every call, whichever
    form runs -- a workspace full of 0xff (a stale flag) must not raise."""
    from mepol_amd import ops

    pol, init, noise = _rollout_inputs("gridworld", [300, 300], 8, 20, 2)
    ref = _rollout_run("gridworld", pol, init, noise)
    for mw in ("0", "1"):
        monkeypatch.setenv("MEPOL_ROLLOUT_MW", mw)
        ops._workspace(torch.device("cuda", 0), 1 << 20, tag="rollout").fill_(0xFF)
        out = _rollout_run("gridworld", pol, init, noise)
        assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])


def test_rollout_under_concurrent_load(cuda, monkeypatch):
    """the multi-workgroup rollout must not depend on having the CUs to itself.  A
    long f64 GEMM queue occupies every CU from another stream while the rollout is launched; the
    result must be the same bits as on an idle GPU (cooperative launch, or the one-workgroup
    fallback, which sums in the same order), with no co-residency error."""
    import warnings

    monkeypatch.setenv("MEPOL_ROLLOUT_MW", "1")
    pol, init, noise = _rollout_inputs("gridworld", [300, 300], 20, 400, 4)
    ref = _rollout_run("gridworld", pol, init, noise)
    a = torch.randn(4096, 4096, dtype=torch.float64, device="cuda")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # a co-residency fallback warning fails the test
        with torch.cuda.stream(side):
            for _ in range(12):  # ~3 ms each: the queue outlasts the rollout's launch
                b = a @ a
        out = _rollout_run("gridworld", pol, init, noise)
        torch.cuda.synchronize()
    del b
    assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])


@pytest.mark.parametrize("env", ["mountaincar", "gridworld"])
@pytest.mark.parametrize("mw", ["1", "0"], ids=["multi-wg", "one-wg"])
@pytest.mark.parametrize("hidden", [[300, 300], [64, 48], [400, 300]])
def test_rollout_mlp_bitexact_vs_kordered_oracle(cuda, monkeypatch, env, mw, hidden):
    """mepol_rollout_mlp against the oracle's k-ordered restatement
    (oracle/native/rollout_kordered.c: the MLP summed in the order the kernels commit to): the
    actions are bit-identical and so are the GridWorld states (f32 state, f64 move: no
    transcendental); MountainCar's cos() may round differently from glibc in the last ulp, so
    its states / actions are checked to 1e-12.  Both kernel forms (ceil(h1/64) workgroups per
    trajectory, MEPOL_ROLLOUT_MW=1, and one workgroup per trajectory) match the oracle in the
    summation order they report (ops.rollout_mlp_plan: k_chunks)."""
    from mepol_amd import ops
    from mepol_amd.policy import GaussianPolicy

    monkeypatch.setenv("MEPOL_ROLLOUT_MW", mw)
    torch.manual_seed(11)
    a_dim = 1 if env == "mountaincar" else 2
    pol = GaussianPolicy(hidden, 2, a_dim, -0.5 if env == "mountaincar" else -1.5).cuda()
    nt, T = 20, 60
    rng = np.random.default_rng(3)
    if env == "mountaincar":
        init = np.stack([rng.uniform(-0.6, -0.4, nt), np.zeros(nt)], 1)
    else:
        init = rng.uniform(-6, -4, (nt, 2)).astype(np.float32)
    noise = rng.standard_normal((T, nt, a_dim))
    sd = {k: v.detach().cpu().numpy() for k, v in pol.state_dict().items()}
    # exp(log_std) as the device computes it (ocml); it agrees with numpy's to an ulp
    std_dev = torch.exp(pol.log_std.detach()).cpu().numpy()
    np.testing.assert_allclose(std_dev, np.exp(sd["log_std"]), rtol=2.3e-16, atol=0)
    plan = ops.rollout_mlp_plan(nt, hidden[0], hidden[1], a_dim)
    assert plan["workgroups_per_traj"] == (1 if mw == "0" or hidden[0] > 306 else
                                           (hidden[1] + 63) // 64)
    S_ref, A_ref = O.rollout_kordered(env, sd, std_dev, init, noise, T, plan["k_chunks"])
    dev = "cuda"
    states = torch.zeros((nt, T + 1, 2), dtype=torch.float32, device=dev)
    actions = torch.zeros((nt, T, a_dim), dtype=torch.float32, device=dev)
    l1, l2 = pol.net[0], pol.net[2]
    ops.rollout_mlp(0 if env == "mountaincar" else 1, l1.weight.detach(), l1.bias.detach(),
                    l2.weight.detach(), l2.bias.detach(), pol.mean.weight.detach(),
                    pol.mean.bias.detach(), pol.log_std.detach(), torch.as_tensor(init, device=dev),
                    torch.as_tensor(noise, dtype=torch.float64, device=dev), states, actions)
    S, A = states.cpu().numpy(), actions.cpu().numpy()
    if env == "gridworld":
        assert np.array_equal(A, A_ref)
        assert np.array_equal(S, S_ref)
    else:
        assert np.array_equal(A[:, 0], A_ref[:, 0])  # first step: no cos() involved yet
        np.testing.assert_allclose(A, A_ref, rtol=0, atol=1e-12)
        np.testing.assert_allclose(S, S_ref, rtol=0, atol=1e-12)
