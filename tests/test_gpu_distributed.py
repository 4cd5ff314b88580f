"""Two ranks sharing one GPU (gloo collectives, HIP kernels) == the single-rank GPU path."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
NT, T, NF, A, K, HID = 8, 250, 29, 8, 30, [64, 48]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    rng = np.random.default_rng(3)
    return (rng.standard_normal((NT, T + 1, NF)).astype(np.float32),
            (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32))


def _consts():
    import scipy.special

    return float(scipy.special.gamma(NF / 2 + 1)), float(np.log(K) - scipy.special.digamma(K))


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist

    from mepol_amd.parallel import ShardedEpoch
    from mepol_amd.policy import GaussianPolicy

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    states, actions = _data()
    per = NT // world
    sl = slice(rank * per, (rank + 1) * per)
    st = torch.as_tensor(states[sl], dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions[sl], dtype=torch.float64, device=dev)
    rtl = torch.full((per, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[sl, 1:].reshape(-1, NF), device=dev)
    torch.manual_seed(1)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    opt = torch.optim.Adam(tgt.parameters(), lr=1e-3)
    G, B = _consts()
    ep = ShardedEpoch(st, ac, rtl, nxt, K, dist)
    ep.build_knn()
    hs, kls = [], []
    for _ in range(3):
        loss, _ = ep.policy_update(opt, beh, tgt, K, G, B, NF, 0.0)
        hs.append(-float(loss))
        kl, _ = ep.compute_kl(beh, tgt, K, 0.0)
        kls.append(float(kl))
    p = torch.cat([q.detach().reshape(-1) for q in tgt.parameters()]).cpu().numpy()
    if rank == 0:
        np.savez(out, hs=hs, kls=kls, params=p, D=ep.D.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_rank(cuda, tmp_path):
    from mepol_amd.algorithms import mepol as M
    from mepol_amd.policy import GaussianPolicy

    out = str(tmp_path / "w2.npz")
    mp.start_processes(_worker, args=(2, _port(), out), nprocs=2, join=True, start_method="spawn")
    r2 = np.load(out)
    states, actions = _data()
    dev = torch.device("cuda:0")
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    torch.manual_seed(1)
    beh = GaussianPolicy(HID, NF, A).to(dev)
    tgt = GaussianPolicy(HID, NF, A).to(dev)
    tgt.load_state_dict(beh.state_dict())
    opt = torch.optim.Adam(tgt.parameters(), lr=1e-3)
    G, B = _consts()
    st_, ac_, rl_, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, K)
    assert np.array_equal(D[: NT // 2 * T].cpu().numpy(), r2["D"])
    hs, kls = [], []
    for _ in range(3):
        loss, _ = M.policy_update(opt, beh, tgt, st_, ac_, NT, rl_, D, I, K, G, B, NF, 0.0)
        hs.append(-float(loss))
        kl, _ = M.compute_kl(beh, tgt, st_, ac_, NT, rl_, D, I, K, 0.0)
        kls.append(float(kl))
    p = torch.cat([q.detach().reshape(-1) for q in tgt.parameters()]).cpu().numpy()
    np.testing.assert_allclose(r2["hs"], hs, rtol=1e-12)
    np.testing.assert_allclose(r2["kls"], kls, rtol=1e-9, atol=1e-14)
    np.testing.assert_allclose(r2["params"], p, rtol=1e-9, atol=1e-12)


class _OneRank:
    """A one-rank stand-in for torch.distributed (ShardedEpoch's collectives are then copies)."""

    def get_world_size(self, group=None):
        return 1

    def get_rank(self, group=None):
        return 0

    def get_backend(self, group=None):
        return "gloo"

    def all_gather_into_tensor(self, out, inp, group=None):
        out.copy_(inp.reshape(-1))

    def all_reduce(self, t, op=None, group=None):
        return None


def test_sharded_knn_rejects_nan(cuda):
    """The sharded epoch reads the k-NN input check after the gather and the CSR build are
    queued: a NaN state must still raise (MepolInputError, a ValueError, as sklearn) and leave
    no partial epoch behind."""
    from mepol_amd._lib import MepolInputError
    from mepol_amd.parallel import ShardedEpoch

    states, actions = _data()
    dev = torch.device("cuda:0")
    st = torch.as_tensor(states, dtype=torch.float64, device=dev)
    ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
    rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
    nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
    bad = nxt.clone()
    bad[7, 1] = float("nan")
    with pytest.raises(MepolInputError):
        ShardedEpoch(st, ac, rtl, bad, K, _OneRank()).build_knn()
    ep = ShardedEpoch(st, ac, rtl, nxt, K, _OneRank())
    D, I = ep.build_knn()
    assert torch.isfinite(D).all()
