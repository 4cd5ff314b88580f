"""Graph-replayed off-policy loop vs the eager loop at a device-loop test shape: prints both
(n, H, KL, lr) traces.  Usage: python tools/loop_debug.py [C3|C4|C5] (env MEPOL_SPECULATE)."""
import os
import sys

import numpy as np
import pytest  # noqa: F401  (tests/ helpers import it)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_device_loop as T  # noqa: E402


class _MP:
    def setenv(self, k, v):
        os.environ[k] = v


cfg = getattr(T, sys.argv[1] if len(sys.argv) > 1 else "C5")
for graph in (True, False):
    g = T._run(_MP(), graph, "adam", 1e-4, 1e9, max_off_iters=3, cfg=cfg)
    print("graph" if graph else "eager", "used", g["used"], "n", g["n"])
    for row in g["trace"]:
        print("   ", row)
