"""Child process of tests/test_gpu_sharded_graph.py: one RCCL process group of world size 1,
the sharded off-policy loop run graph-replayed and eagerly for each case, then the teardown
the CLI uses (parallel.destroy_process_group).  Writes the traces to argv[1] as JSON."""
import json
import os
import socket
import sys

import numpy as np
import scipy.special
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]
CASES = [(10.0, 1e-3), (1e-3, 5e-2)]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(dist, graph, kl_threshold, lr):
    from mepol_amd import parallel
    from mepol_amd.parallel import ShardedEpoch
    from mepol_amd.policy import GaussianPolicy

    os.environ["MEPOL_DEVICE_LOOP"] = "1" if graph else "0"
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
    return dict(H=float(res[0]), n=res[1], bt=res[2], lr=res[3], trace=trace,
                params=p.tolist(), graph=it is not None and it.graph is not None)


def main():
    import torch.distributed as dist

    from mepol_amd import parallel

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_port())
    os.environ["MEPOL_CHECK_RANKS"] = "1"  # the debug cross-rank (H, KL) agreement check
    torch.cuda.set_device(0)
    parallel.prepare_nccl_env()  # as the CLI and bench.py do before init_process_group
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    out = {}
    for i, (kl, lr) in enumerate(CASES):
        out[str(i)] = dict(graph=_run(dist, True, kl, lr), eager=_run(dist, False, kl, lr))
        print(f"case {i} done", flush=True)
    parallel.destroy_process_group(dist)
    out["released"] = len(parallel._SHARDED_CACHE)
    with open(sys.argv[1], "w") as f:
        json.dump(out, f)
    print("worker ok", flush=True)


if __name__ == "__main__":
    main()
