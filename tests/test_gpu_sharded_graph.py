"""The sharded off-policy iteration replayed as one graph with its RCCL collectives captured
(parallel.ShardedIteration) == the eager sharded path == the single-rank path.  World size 1
over the nccl (RCCL) backend on the box's one GPU: the capture, the collectives inside the graph
and the consensus logic run for real; the multi-rank algebra itself is covered by the gloo tests."""
import os
import socket

import numpy as np
import pytest
import scipy.special
import torch

pytestmark = pytest.mark.gpu

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_world1():
    import torch.distributed as dist

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    torch.cuda.set_device(0)
    from mepol_amd.parallel import prepare_nccl_env

    prepare_nccl_env()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    yield dist
    dist.destroy_process_group()


def _run(dist, graph, monkeypatch, kl_threshold=10.0, lr=1e-3):
    from mepol_amd import parallel
    from mepol_amd.parallel import ShardedEpoch
    from mepol_amd.policy import GaussianPolicy

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    rng = np.random.default_rng(7)
    states = rng.standard_normal((NT, T + 1, NF)).astype(np.float32)
    actions = (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32)
    dev = torch.device("cuda:0")
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    torch.manual_seed(7)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    last = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    last.load_state_dict(beh.state_dict())
    opt = torch.optim.Adam(tgt.parameters(), lr=lr)
    G = float(scipy.special.gamma(NF / 2 + 1))
    B = float(np.log(K) - scipy.special.digamma(K))
    ep = ShardedEpoch(st, ac, rtl, nxt, K, dist)
    ep.build_knn()
    trace = []
    res = ep.off_policy_optimization(opt, beh, tgt, last, G, B, NF, 0.0, kl_threshold, 6, True,
                                     2, 4, lr, on_accept=lambda n, e, kl, l: trace.append(
                                         (n, float(e), float(kl), l)))
    it = parallel._SHARDED_CACHE.get(tgt)
    p = torch.cat([q.detach().reshape(-1) for q in last.parameters()]).cpu().numpy()
    return dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace, params=p,
                graph=it is not None and it.graph is not None)


@pytest.mark.parametrize("kl_threshold,lr", [(10.0, 1e-3), (1e-3, 5e-2)])
def test_sharded_graph_matches_eager(cuda, nccl_world1, monkeypatch, kl_threshold, lr):
    monkeypatch.setenv("MEPOL_CHECK_RANKS", "1")  # the debug cross-rank (H, KL) agreement check
    g = _run(nccl_world1, True, monkeypatch, kl_threshold, lr)
    e = _run(nccl_world1, False, monkeypatch, kl_threshold, lr)
    assert g["graph"], "the sharded iteration was not captured"
    assert not e["graph"]
    assert (g["n"], g["bt"], g["lr"]) == (e["n"], e["bt"], e["lr"])
    assert len(g["trace"]) == len(e["trace"])
    assert len(g["trace"]) > 0 or kl_threshold < 1  # the tiny threshold rejects every step
    for a, b in zip(g["trace"], e["trace"]):
        assert a[0] == b[0] and a[3] == b[3]
        np.testing.assert_allclose(a[1:3], b[1:3], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(g["H"], e["H"], rtol=1e-9)
    np.testing.assert_allclose(g["params"], e["params"], rtol=1e-8, atol=1e-11)
