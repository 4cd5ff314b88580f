"""The graph-replayed sharded iteration at world size 2, in one process (the multi-rank
layout of parallel.ShardedIteration -- the CSR remap j // n * (n + 4), the (n + nt) block stride
of iw_normalize_gathered, the gathered S partials of the reverse scan, the two-bucket gradient
all-reduce -- was only ever replayed at world 1, where all of it is the identity).

_TwinDist is a world-2 "group" whose second rank holds an exact copy of the first rank's
shard.  Every payload rank 1 would contribute is then bit-identical to rank 0's: its k-NN rows
(the candidate set and every distance are the same for twins, ties go to the smaller index on
both), its weights, dH/dW and block partials, its gradient.  So all_gather = rank 0's payload
in both slots and all_reduce(SUM) = 2 x rank 0's values (exact) reproduce a real 2-rank job on
that data, with the peer's blocks at their real offsets.  The collectives are copy kernels, so
the graph path captures them like RCCL ones (get_backend() says "nccl").

Checked: graph replay == eager sharded path (trace, H, parameters) and both == the single-rank
path (one GPU, no sharding) over the duplicated dataset; csr_rows_x == an explicit per-rank map."""
import os

import numpy as np
import pytest
import scipy.special
import torch

pytestmark = pytest.mark.gpu

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]  # >= 16384 rows per rank: fused path
CASES = [(10.0, 1e-3), (1e-3, 5e-2)]


class _TwinDist:
    class ReduceOp:
        SUM, MIN, MAX = "sum", "min", "max"

    world = 2

    def get_world_size(self, group=None):
        return self.world

    def get_rank(self, group=None):
        return 0

    def get_backend(self, group=None):
        return "nccl"

    def all_gather_into_tensor(self, out, inp, group=None):
        out.view(self.world, -1).copy_(inp.reshape(1, -1).expand(self.world, -1))

    def all_reduce(self, t, op="sum", group=None):
        if op == self.ReduceOp.SUM:
            t.mul_(self.world)  # x + x, exactly

    def barrier(self, group=None):
        pass


def _data():
    rng = np.random.default_rng(11)
    return (rng.standard_normal((NT, T + 1, NF)).astype(np.float32),
            (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32))


def _policies(dev, lr):
    from mepol_amd.policy import GaussianPolicy

    torch.manual_seed(5)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    last = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    last.load_state_dict(beh.state_dict())
    return beh, tgt, last, torch.optim.Adam(tgt.parameters(), lr=lr)


def _consts():
    return float(scipy.special.gamma(NF / 2 + 1)), float(np.log(K) - scipy.special.digamma(K))


def _result(res, trace, last):
    p = torch.cat([q.detach().reshape(-1) for q in last.parameters()]).cpu().numpy()
    return dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace, params=p)


def _sharded(graph, kl_threshold, lr, monkeypatch):
    from mepol_amd import parallel
    from mepol_amd.parallel import ShardedEpoch

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1" if graph else "0")
    dev = torch.device("cuda:0")
    states, actions = _data()
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    beh, tgt, last, opt = _policies(dev, lr)
    G, B = _consts()
    ep = ShardedEpoch(st, ac, rtl, nxt, K, _TwinDist())
    ep.build_knn()
    trace = []
    res = ep.off_policy_optimization(opt, beh, tgt, last, G, B, NF, 0.0, kl_threshold, 6, True, 2,
                                     4, lr, on_accept=lambda n, e, kl, l: trace.append(
                                         (n, float(e), float(kl), l)))
    it = parallel._SHARDED_CACHE.get(tgt)
    out = _result(res, trace, last)
    out["graph"] = it is not None and it.graph is not None
    if out["graph"]:
        n = NT * T
        rows = it.csr_rows.long().cpu()
        expect = rows // n * (n + 4) + rows % n
        out["csr_remap_ok"] = bool(torch.equal(it.csr_rows_x.long().cpu(), expect))
        out["peer_rows"] = int((rows >= n).sum())
    parallel.release_graphs()
    return out


def _single_rank(kl_threshold, lr, monkeypatch):
    """One rank, no sharding, over the duplicated dataset (rank 1's trajectories after rank
    0's, the reference's traj-major order)."""
    from mepol_amd.algorithms import mepol as M

    monkeypatch.setenv("MEPOL_DEVICE_LOOP", "1")
    dev = torch.device("cuda:0")
    states, actions = _data()
    states, actions = np.concatenate([states, states]), np.concatenate([actions, actions])
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((2 * NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    beh, tgt, last, opt = _policies(dev, lr)
    G, B = _consts()
    st_, ac_, rl_, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, K)
    trace = []
    res = M.off_policy_optimization(opt, beh, tgt, last, st_, ac_, 2 * NT, rl_, D, I, K, G, B, NF,
                                    0.0, kl_threshold, 6, True, 2, 4, lr,
                                    on_accept=lambda n, e, kl, l: trace.append(
                                        (n, float(e), float(kl), l)))
    return _result(res, trace, last)


def _same(a, b, rtol):
    assert (a["n"], a["bt"], a["lr"]) == (b["n"], b["bt"], b["lr"])
    assert len(a["trace"]) == len(b["trace"])
    for x, y in zip(a["trace"], b["trace"]):
        assert x[0] == y[0] and x[3] == y[3]
        np.testing.assert_allclose(x[1:3], y[1:3], rtol=rtol, atol=1e-12)
    np.testing.assert_allclose(a["H"], b["H"], rtol=rtol)
    np.testing.assert_allclose(a["params"], b["params"], rtol=1e-8, atol=1e-11)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sharded_graph_world2_matches_eager_and_single_rank(cuda, monkeypatch, case):
    kl_threshold, lr = CASES[case]
    g = _sharded(True, kl_threshold, lr, monkeypatch)
    e = _sharded(False, kl_threshold, lr, monkeypatch)
    s = _single_rank(kl_threshold, lr, monkeypatch)
    assert g["graph"], "the sharded iteration was not captured"
    assert g["csr_remap_ok"] and g["peer_rows"] > 0  # neighbours in rank 1's block, remapped
    assert len(g["trace"]) > 0 or kl_threshold < 1   # the tiny threshold rejects every step
    _same(g, e, 1e-9)
    _same(g, s, 1e-9)
