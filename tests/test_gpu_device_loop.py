"""The graph-replayed off-policy iteration (algorithms/device_loop.py) == the eager path
(autograd through the same kernels) == the oracle's torch CPU loop, with Adam and RMSprop,
with and without backtracking (mepol.py:416-483)."""
import copy

import numpy as np
import pytest
import scipy.special
import torch

pytestmark = pytest.mark.gpu

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]  # N = 20000 >= the fused-path minimum
SMALL = dict(NT=NT, T=T, NF=NF, A=A, K=K, HID=HID)
# The BASELINE policy/k shapes (ANT, HUM, HR) at N = 20000 particles
C3 = dict(NT=40, T=500, NF=29, A=8, K=30, HID=[400, 300])
C4 = dict(NT=40, T=500, NF=47, A=17, K=30, HID=[400, 300])
C5 = dict(NT=400, T=50, NF=63, A=20, K=50, HID=[400, 300])
# the full BASELINE batches the bench runs (C3: 400 x 500 = 200k particles; C5: 10000 x 50 =
# 500k particles)
C3_FULL = dict(NT=400, T=500, NF=29, A=8, K=30, HID=[400, 300])
C5_FULL = dict(NT=10000, T=50, NF=63, A=20, K=50, HID=[400, 300])


def _setup(opt_name, lr, seed=5, cfg=None):
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.policy import GaussianPolicy

    c = cfg or SMALL
    NT, T, NF, A, K, HID = c["NT"], c["T"], c["NF"], c["A"], c["K"], c["HID"]
    rng = np.random.default_rng(seed)
    states = rng.standard_normal((NT, T + 1, NF)).astype(np.float32)
    actions = (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32)
    dev = torch.device("cuda")
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    torch.manual_seed(seed)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    last = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    last.load_state_dict(beh.state_dict())
    opt_cls = torch.optim.Adam if opt_name == "adam" else torch.optim.RMSprop
    opt = opt_cls(tgt.parameters(), lr=lr)
    batch = M.make_particle_batch(st, ac, rtl, nxt, K)
    return M, (states, actions), beh, tgt, last, opt, batch


def _run(monkeypatch, graph, opt_name, lr, kl_threshold, max_off_iters=6, cfg=None,
         backtracking=True):
    from mepol_amd.algorithms import device_loop

    c = cfg or SMALL
    NT, NF, K = c["NT"], c["NF"], c["K"]
    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    M, raw, beh, tgt, last, opt, (st, ac, rl, _, D, I) = _setup(opt_name, lr, cfg=c)
    G = float(scipy.special.gamma(NF / 2 + 1))
    B = float(np.log(K) - scipy.special.digamma(K))
    trace = []
    res = M.off_policy_optimization(
        opt, beh, tgt, last, st, ac, NT, rl, D, I, K, G, B, NF, 0.0, kl_threshold, max_off_iters,
        backtracking, 2, 4, lr,
        on_accept=lambda n, e, kl, l: trace.append((n, float(e), float(kl), l)))
    used = tgt in device_loop._CACHE
    it = device_loop._CACHE.get(tgt)
    fused = (it.fused_fwd, it.fused_dh1) if it is not None else None
    params = torch.cat([p.detach().reshape(-1) for p in last.parameters()]).cpu().numpy()
    state = opt.state_dict()["state"]
    steps = [float(state[i]["step"]) for i in sorted(state)]
    moments = np.concatenate([state[i][key].detach().reshape(-1).cpu().numpy()
                              for i in sorted(state) for key in sorted(state[i])
                              if key != "step"])
    tparams = torch.cat([p.detach().reshape(-1) for p in tgt.parameters()]).cpu().numpy()
    return dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace, params=params,
                steps=steps, used=used, raw=raw, D=D, I=I, moments=moments, tparams=tparams,
                fused=fused)


def _assert_same_run(g, e):
    assert g["used"] and not e["used"]
    assert (g["n"], g["bt"], g["lr"]) == (e["n"], e["bt"], e["lr"])
    assert g["steps"] == e["steps"]
    assert len(g["trace"]) == len(e["trace"])
    for a, b in zip(g["trace"], e["trace"]):
        assert a[0] == b[0] and a[3] == b[3]
        np.testing.assert_allclose(a[1:3], b[1:3], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(g["H"], e["H"], rtol=1e-9)
    np.testing.assert_allclose(g["params"], e["params"], rtol=1e-8, atol=1e-11)
    np.testing.assert_allclose(g["tparams"], e["tparams"], rtol=1e-8, atol=1e-11)
    # the optimizer moments carry into the next epoch: a cancelled speculative replay must
    # leave them exactly as the rejected step did
    np.testing.assert_allclose(g["moments"], e["moments"], rtol=1e-8, atol=1e-14)


@pytest.mark.parametrize("opt_name,lr,kl_threshold,cfg", [
    ("adam", 1e-3, 10.0, SMALL),     # all steps accepted until max_off_iters
    ("adam", 5e-2, 1e-3, SMALL),     # early rejection -> backtracking with halved lr
    ("rmsprop", 1e-4, 10.0, SMALL),
    ("adam", 1e-4, 10.0, C4),        # wide action head (a = 17)
])
def test_graph_loop_matches_eager(cuda, monkeypatch, opt_name, lr, kl_threshold, cfg):
    g = _run(monkeypatch, True, opt_name, lr, kl_threshold, cfg=cfg)
    e = _run(monkeypatch, False, opt_name, lr, kl_threshold, cfg=cfg)
    _assert_same_run(g, e)


@pytest.mark.parametrize("backtracking", [True, False])
@pytest.mark.parametrize("speculate", ["1", "0"])
def test_graph_loop_mid_loop_rejection(cuda, monkeypatch, backtracking, speculate):
    """A step rejected after accepted ones, while the next replay is already in flight
    (speculative launch): the cancelled replay leaves theta, the moments and the step count
    as the eager loop does, with and without backtracking."""
    monkeypatch.setenv("MEPOL_SPECULATE", speculate)
    probe = _run(monkeypatch, False, "adam", 1e-3, 1e9, max_off_iters=6)
    kls = [t[2] for t in probe["trace"]]
    # the last step whose KL exceeds every earlier one: a threshold between them accepts the
    # steps before it and rejects it (KL is not monotone in the step count)
    cut = [i for i in range(1, len(kls)) if kls[i] > max(kls[:i])]
    assert len(kls) == 6 and cut, kls
    i = cut[-1]
    thr = 0.5 * (max(kls[:i]) + kls[i])
    g = _run(monkeypatch, True, "adam", 1e-3, thr, max_off_iters=6, backtracking=backtracking)
    e = _run(monkeypatch, False, "adam", 1e-3, thr, max_off_iters=6, backtracking=backtracking)
    assert i <= e["n"] <= i + int(backtracking)  # + the backtracked step, if accepted
    _assert_same_run(g, e)


def _oracle_steps(g, cfg, lr, steps):
    """Replay `steps` accepted Adam steps of the oracle's torch-CPU policy_update/compute_kl
    (oracle/mepol_oracle.py, mepol.py:268-281, 157-174) from _setup's initial weights on the
    same particles and the GPU's D/I; compare H, KL per step and the final parameters."""
    import oracle.mepol_oracle as O
    from mepol_amd.policy import GaussianPolicy

    NT, T, NF, A, K, HID = cfg["NT"], cfg["T"], cfg["NF"], cfg["A"], cfg["K"], cfg["HID"]
    states, actions = g["raw"]
    torch.manual_seed(5)
    sd = GaussianPolicy(HID, NF, A).state_dict()  # the initial weights _setup drew
    beh = O.TorchPolicy(HID, NF, A)
    beh.load_state_dict(sd)
    tgt = copy.deepcopy(beh)
    opt = torch.optim.Adam(tgt.parameters(), lr=lr)
    S = torch.as_tensor(states, dtype=torch.float64)
    Ac = torch.as_tensor(actions, dtype=torch.float64)
    lengths = torch.full((NT, 1), T, dtype=torch.int64)
    D, I = g["D"].cpu(), g["I"].cpu()
    G = float(scipy.special.gamma(NF / 2 + 1))
    B = float(np.log(K) - scipy.special.digamma(K))
    for it in range(steps):
        loss, _ = O.torch_policy_update(opt, beh, tgt, S, Ac, NT, lengths, D, I, K, G, B, NF, 0.0)
        kl, _ = O.torch_kl(beh, tgt, S, Ac, NT, lengths, I, K, 0.0)
        np.testing.assert_allclose(g["trace"][it][1], -float(loss.detach()), rtol=1e-9)
        np.testing.assert_allclose(g["trace"][it][2], float(kl), rtol=1e-9, atol=1e-13)
    p = torch.cat([q.detach().reshape(-1) for q in tgt.parameters()]).numpy()
    np.testing.assert_allclose(g["params"], p, rtol=1e-7, atol=1e-10)


@pytest.mark.parametrize("cfg,lr", [(SMALL, 1e-3), (C3, 1e-4), (C4, 1e-4), (C5, 1e-4)],
                         ids=["small", "C3-shape", "C4-shape", "C5-shape"])
def test_graph_loop_matches_oracle(cuda, monkeypatch, cfg, lr):
    """Three accepted Adam steps against the oracle's torch-CPU policy_update/compute_kl, at the
    BASELINE policy shapes (29/47/63 -> [400, 300] -> 8/17/20, k = 30/30/50; N = 20000)."""
    g = _run(monkeypatch, True, "adam", lr, 1e9, max_off_iters=3, cfg=cfg)
    assert g["used"] and g["n"] == 3
    _oracle_steps(g, cfg, lr, 3)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,steps", [(C3_FULL, 2), (C5_FULL, 1)], ids=["C3", "C5"])
def test_graph_loop_matches_oracle_full_size(cuda, monkeypatch, cfg, steps):
    """the graph-replayed iteration at the benchmarked sizes (C3 N = 200k,
    d = 29, k = 30; C5 N = 500k, d = 63, k = 50) against the oracle's torch-CPU step."""
    g = _run(monkeypatch, True, "adam", 1e-4, 1e9, max_off_iters=steps, cfg=cfg)
    assert g["used"] and g["n"] == steps
    _oracle_steps(g, cfg, 1e-4, steps)


def _two_epochs(monkeypatch, graph):
    """Two off-policy loops on one batch with an eager backward on a larger batch in between
    (it grows the eager scratch cache while the first loop's graph is kept for the second)."""
    from mepol_amd.policy import GaussianPolicy

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    M, raw, beh, tgt, last, opt, (st, ac, rl, _, D, I) = _setup("adam", 1e-3)
    G = float(scipy.special.gamma(NF / 2 + 1))
    B = float(np.log(K) - scipy.special.digamma(K))
    out = []
    for epoch in range(2):
        res = M.off_policy_optimization(opt, beh, tgt, last, st, ac, NT, rl, D, I, K, G, B, NF,
                                        0.0, 1e9, 2, True, 2, 4, 1e-3)
        out.append(float(res[0]))
        beh.load_state_dict(last.state_dict())
        tgt.load_state_dict(last.state_dict())
        if epoch == 0:
            big = GaussianPolicy(HID, NF, A).cuda()
            s = torch.randn(3 * NT * T, NF, dtype=torch.float64, device="cuda")
            a = torch.randn(3 * NT * T, A, dtype=torch.float64, device="cuda")
            big.get_log_p(s, a).sum().backward()
    from mepol_amd.algorithms import device_loop

    params = torch.cat([p.detach().reshape(-1) for p in last.parameters()]).cpu().numpy()
    import weakref

    return out, params, (tgt in device_loop._CACHE, weakref.ref(tgt))


def test_graph_scratch_survives_eager_growth(cuda, monkeypatch):
    """a captured iteration must not write through scratch the eager path replaced."""
    from mepol_amd.algorithms import device_loop

    g_out, g_params, (used, tgt_ref) = _two_epochs(monkeypatch, True)
    assert used
    # the cache is keyed weakly by the target policy and its entry does not keep it alive:
    # once the caller's policy is gone, so is the graph with its ~N-sized static buffers
    import gc

    gc.collect()
    assert tgt_ref() is None
    e_out, e_params, _ = _two_epochs(monkeypatch, False)
    np.testing.assert_allclose(g_out, e_out, rtol=1e-9)
    np.testing.assert_allclose(g_params, e_params, rtol=1e-8, atol=1e-11)


def _fresh_batch_epochs(monkeypatch, graph, thr):
    """epoch 1 ends on a rejected step (no backtracking), epoch 2 runs on a
    different batch of the same shape: the cached graph must take its activations from the new
    batch at the new behavioral parameters, not from epoch 1's last (rejected) replay."""
    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    M, _, beh, tgt, last, opt, b1 = _setup("adam", 1e-3, seed=5)
    b2 = _setup("adam", 1e-3, seed=6)[-1]
    G = float(scipy.special.gamma(NF / 2 + 1))
    Bc = float(np.log(K) - scipy.special.digamma(K))
    out = []
    for (st, ac, rl, _, D, I), t in ((b1, thr), (b2, 1e9)):
        trace = []
        res = M.off_policy_optimization(
            opt, beh, tgt, last, st, ac, NT, rl, D, I, K, G, Bc, NF, 0.0, t, 6, False, 2, 4,
            1e-3, on_accept=lambda n, e, kl, l: trace.append((n, float(e), float(kl))))
        out.append((float(res[0]), res[1], trace))
        beh.load_state_dict(last.state_dict())
        tgt.load_state_dict(last.state_dict())
    state = opt.state_dict()["state"]
    moments = np.concatenate([state[i][key].detach().reshape(-1).cpu().numpy()
                              for i in sorted(state) for key in sorted(state[i])
                              if key != "step"])
    params = torch.cat([p.detach().reshape(-1) for p in last.parameters()]).cpu().numpy()
    return out, params, moments


def test_graph_loop_fresh_batch_after_rejection(cuda, monkeypatch):
    probe = _run(monkeypatch, False, "adam", 1e-3, 1e9, max_off_iters=6)
    kls = [t[2] for t in probe["trace"]]
    cut = [i for i in range(1, len(kls)) if kls[i] > max(kls[:i])]
    assert cut, kls
    i = cut[-1]
    thr = 0.5 * (max(kls[:i]) + kls[i])
    g_out, g_params, g_mom = _fresh_batch_epochs(monkeypatch, True, thr)
    e_out, e_params, e_mom = _fresh_batch_epochs(monkeypatch, False, thr)
    assert g_out[0][1] == e_out[0][1] == i  # epoch 1: i accepted steps, then the rejection
    for (gH, gn, gt), (eH, en, et) in zip(g_out, e_out):
        assert gn == en and len(gt) == len(et)
        np.testing.assert_allclose(gH, eH, rtol=1e-9)
        for a, b in zip(gt, et):
            np.testing.assert_allclose(a[1:], b[1:], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(g_params, e_params, rtol=1e-8, atol=1e-11)
    np.testing.assert_allclose(g_mom, e_mom, rtol=1e-8, atol=1e-14)


@pytest.mark.parametrize("fwd,dh1", [("0", "1"), ("1", "0"), ("0", "0")])
def test_unfused_mlp_kernels_match_fused(cuda, monkeypatch, fwd, dh1):
    """MEPOL_FUSED_FWD=0 / MEPOL_FUSED_DH1=0 select the unfused forward (layer kernels + GEMM)
    and backward (dh1 GEMM + separate layer-1 backward) inside the captured iteration, the form
    used where the fused kernels' shape limits are not met; both forms agree with each other."""
    ref = _run(monkeypatch, True, "adam", 1e-4, 1e9, max_off_iters=3, cfg=C3)
    monkeypatch.setenv("MEPOL_FUSED_FWD", fwd)
    monkeypatch.setenv("MEPOL_FUSED_DH1", dh1)
    got = _run(monkeypatch, True, "adam", 1e-4, 1e9, max_off_iters=3, cfg=C3)
    assert got["used"] and ref["used"] and got["n"] == ref["n"] == 3
    assert ref["fused"] == (True, True) and got["fused"] == (fwd == "1", dh1 == "1")
    for a, b in zip(got["trace"], ref["trace"]):
        np.testing.assert_allclose(a[1:3], b[1:3], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(got["params"], ref["params"], rtol=1e-8, atol=1e-11)
