"""Multi-rank particle sharding (mepol_amd/parallel.py) on CPU with the gloo backend.

World sizes 1 and 2 run the same global batch through ShardedEpoch (collectives real, kernels
replaced by the CPU stand-ins of tests/cpu_ops.py); they must agree with each other and with the
oracle's single-process closed forms, and every rank must end with identical parameters.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


NT, T, NF, A, K, HID = 4, 30, 5, 2, 6, [16, 12]


def _global_batch():
    rng = np.random.default_rng(0)
    states = rng.standard_normal((NT, T + 1, NF)).astype(np.float32)
    actions = (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32)
    return states, actions


def _worker(rank, world, port, out_path):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import scipy.special
    import torch.distributed as dist

    import cpu_ops
    from mepol_amd.parallel import ShardedEpoch
    from mepol_amd.policy import GaussianPolicy

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    states, actions = _global_batch()
    per = NT // world
    st = torch.as_tensor(states[rank * per:(rank + 1) * per], dtype=torch.float64)
    ac = torch.as_tensor(actions[rank * per:(rank + 1) * per], dtype=torch.float64)
    rtl = torch.full((per, 1), T, dtype=torch.int64)
    nxt = torch.as_tensor(states[rank * per:(rank + 1) * per, 1:].reshape(-1, NF))
    torch.manual_seed(1)
    beh = GaussianPolicy(HID, NF, A)
    tgt = GaussianPolicy(HID, NF, A)
    lv = GaussianPolicy(HID, NF, A)
    tgt.load_state_dict(beh.state_dict())
    lv.load_state_dict(beh.state_dict())
    opt = torch.optim.Adam(tgt.parameters(), lr=1e-2)
    ep = ShardedEpoch(st, ac, rtl, nxt, K, dist, ops=cpu_ops)
    ep.build_knn()
    B = float(np.log(K) - scipy.special.digamma(K))
    G = float(scipy.special.gamma(NF / 2 + 1))
    hs, kls, grads = [], [], []
    for it in range(3):
        loss, err = ep.policy_update(opt, beh, tgt, K, G, B, NF, 0.0)
        hs.append(-float(loss))
        grads.append(torch.cat([p.grad.reshape(-1) for p in tgt.parameters()]).numpy().copy())
        kl, kerr = ep.compute_kl(beh, tgt, K, 0.0)
        kls.append(float(kl))
    # the full control loop too (accept/backtrack path must agree across ranks)
    res = ep.off_policy_optimization(opt, beh, tgt, lv, G, B, NF, 0.0, 15.0, 4, True, 2, 10, 1e-2)
    params = torch.cat([p.detach().reshape(-1) for p in tgt.parameters()]).numpy()
    all_params = [torch.zeros_like(torch.as_tensor(params)) for _ in range(world)]
    dist.all_gather(all_params, torch.as_tensor(params))
    if rank == 0:
        np.savez(out_path, hs=np.array(hs), kls=np.array(kls), grads=np.stack(grads),
                 params=params, final_H=float(res[0]), n_off=res[1],
                 rank_params=np.stack([p.numpy() for p in all_params]),
                 D=ep.D.numpy(), I=ep.I.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _run(world, tmp_path):
    out = str(tmp_path / f"w{world}.npz")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    return np.load(out)


@pytest.fixture(scope="module")
def results(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("gloo")
    return _run(1, tmp), _run(2, tmp)


def test_two_ranks_match_one_rank(results):
    r1, r2 = results
    np.testing.assert_allclose(r2["hs"], r1["hs"], rtol=1e-12)
    np.testing.assert_allclose(r2["kls"], r1["kls"], rtol=1e-10, atol=1e-15)
    np.testing.assert_allclose(r2["grads"], r1["grads"], rtol=1e-9, atol=1e-13)
    np.testing.assert_allclose(r2["params"], r1["params"], rtol=1e-9, atol=1e-12)
    assert int(r2["n_off"]) == int(r1["n_off"])
    np.testing.assert_allclose(float(r2["final_H"]), float(r1["final_H"]), rtol=1e-12)


def test_ranks_hold_identical_parameters(results):
    _, r2 = results
    rp = r2["rank_params"]
    assert np.array_equal(rp[0], rp[1])


def test_one_rank_matches_oracle_closed_form(results):
    """ShardedEpoch(world=1) iteration 0 == the oracle's single-process H and gradient."""
    sys.path.insert(0, ROOT)
    from oracle import mepol_oracle as O

    r1, _ = results
    import scipy.special

    states, actions = _global_batch()
    torch.manual_seed(1)
    from mepol_amd.policy import GaussianPolicy

    beh = GaussianPolicy(HID, NF, A)
    sd = {k: v.numpy() for k, v in beh.state_dict().items()}
    nxt = states[:, 1:].reshape(-1, NF)
    D, I = O.knn_exact(nxt, K + 1)
    assert np.array_equal(D[: len(r1["D"])], r1["D"])
    w = np.full(NT * T, 1.0 / (NT * T))  # target == behavioral at iteration 0
    B = float(np.log(K) - scipy.special.digamma(K))
    G = float(scipy.special.gamma(NF / 2 + 1))
    H = O.entropy(w, D, I, K, G, B, NF, 0.0)
    assert abs(H - r1["hs"][0]) <= 1e-12 * abs(H)
    c = O.entropy_grad_logp(w, D, I, K, G, NF, 0.0, [T] * NT)
    ref = GaussianPolicy(HID, NF, A)
    ref.load_state_dict(beh.state_dict())
    S = torch.as_tensor(states, dtype=torch.float64)
    Ac = torch.as_tensor(actions, dtype=torch.float64)
    lp = ref.get_log_p(S[:, :T].reshape(NT * T, NF), Ac.reshape(NT * T, A)).reshape(NT, T)
    (-(torch.as_tensor(c) * lp).sum()).backward()
    g = torch.cat([p.grad.reshape(-1) for p in ref.parameters()]).numpy()
    np.testing.assert_allclose(r1["grads"][0], g, rtol=1e-9, atol=1e-13)
