"""The sharded off-policy iteration replayed as one graph with its RCCL collectives captured
(parallel.ShardedIteration) == the eager sharded path == the single-rank path.  World size 1
over the nccl (RCCL) backend on the box's one GPU: the capture, the collectives inside the graph
and the consensus logic run for real; the multi-rank algebra itself is covered by the gloo tests.

The RCCL process group lives in a child process (tests/sharded_graph_worker.py): its lifetime
(init -> eager collectives -> capture -> speculative replays -> teardown) is exactly a CLI run's,
and a native failure in any RCCL / ProcessGroupNCCL thread fails this test with the child's
stderr instead of aborting the whole GPU suite."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [(10.0, 1e-3), (1e-3, 5e-2)]


@pytest.fixture(scope="module")
def worker_results(cuda, tmp_path_factory):
    out = str(tmp_path_factory.mktemp("sharded") / "res.json")
    env = dict(os.environ)
    cmd = [sys.executable, "-u", os.path.join(HERE, "sharded_graph_worker.py"), out]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    tail = (p.stdout[-3000:] + "\n--- stderr ---\n" + p.stderr[-6000:])
    assert p.returncode == 0, f"worker exited with {p.returncode}:\n{tail}"
    with open(out) as f:
        return json.load(f)


@pytest.mark.parametrize("case", range(len(CASES)))
def test_sharded_graph_matches_eager(worker_results, case):
    kl_threshold, _ = CASES[case]
    g, e = worker_results[str(case)]["graph"], worker_results[str(case)]["eager"]
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


def test_process_group_teardown_released_graphs(worker_results):
    """destroy_process_group ran after parallel.release_graphs() freed every captured graph."""
    assert worker_results["released"] == 0
