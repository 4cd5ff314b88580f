"""bench.py --gpus N without a launcher spawns N rank processes (the flag was
ignored).  CPU-only: the --selftest path runs the real spawn / rendezvous / max-over-ranks
timing over gloo and rank 0 prints the one JSON line with n_gpus = N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_ranks(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                          "--steps", "3", "--selftest"], capture_output=True, text=True,
                         timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["selftest"]
    # every rank took part in every all-reduce: (1 + ... + n) * n^(steps - 1)
    assert rec["sum_of_ranks"] == (n * (n + 1) / 2) * n ** 2


def test_bench_workloads_parse():
    sys.path.insert(0, ROOT)
    import bench

    for w in ("C2", "C2S", "C3", "C4", "C5", "C3R8", "C4R8", "C5R8"):
        cfg = bench.WORKLOADS[w]
        assert cfg["num_traj"] % 8 == 0 or w.startswith("C2")
        args = bench.parse(["--workload", w, "--gpus", "2"])
        assert args.workload == w and args.gpus == 2


def test_emulated_dist_fills_peer_slots():
    """The R8 workloads run rank 0 of an 8-rank job on one GPU: every collective becomes local
    copies of the same size; gathers take registered peer tensors (the other shards' next states,
    so the k-NN sees all N candidates) or replicate rank 0's payload."""
    import torch

    sys.path.insert(0, ROOT)
    import bench

    d = bench._EmulatedDist(4)
    assert d.get_world_size() == 4 and d.get_rank() == 0 and d.get_backend() == "nccl"
    own = torch.arange(6, dtype=torch.float32).reshape(3, 2)
    d.peers = [torch.full((3, 2), float(r)) for r in (1, 2, 3)]
    out = torch.empty(4 * 6, dtype=torch.float32)
    d.all_gather_into_tensor(out, own.reshape(-1))    # ShardedEpoch passes flattened payloads
    o = out.view(4, 3, 2)
    assert torch.equal(o[0], own) and all(bool((o[r] == r).all()) for r in (1, 2, 3))
    w = torch.arange(5, dtype=torch.float64)
    outw = torch.empty(20, dtype=torch.float64)
    d.all_gather_into_tensor(outw, w)            # no peer of this shape: rank 0's payload
    assert torch.equal(outw.view(4, 5), w.expand(4, 5))
    g = torch.ones(3, dtype=torch.float64)
    d.all_reduce(g)
    assert torch.equal(g, torch.ones(3, dtype=torch.float64))
