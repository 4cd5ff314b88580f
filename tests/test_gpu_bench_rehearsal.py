"""bench.py --gpus 2 end to end on the box's one GPU: the launcher spawns two
rank processes, they share the GPU over gloo (the line says "rehearsal"), run the sharded epoch
(ShardedEpoch: next-state all-gather, query-sharded k-NN, per-iteration reductions) and rank 0
prints one JSON line with the max-over-ranks clock and one k-NN time per rank."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_rank_rehearsal(cuda):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--workload", "C3", "--steps", "1", "--warmup", "0",
                          "--no-cpu-baseline"], capture_output=True, text=True, timeout=280,
                         env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 1
    assert len(rec["knn_ms_per_rank"]) == 2 and all(x > 0 for x in rec["knn_ms_per_rank"])
    assert rec["config"]["parallelism"] == "dp2"
    assert "rehearsal" in rec["config"]
    assert rec["value"] > 0 and rec["config"]["off_policy_iters"] >= 1
