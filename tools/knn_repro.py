"""k-NN determinism / exactness at the device-loop test's C5 shape (N = 20000, d = 63, k+1 = 51):
three calls per split setting, compared with each other and with the oracle's exhaustive scan."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mepol_amd import ops  # noqa: E402
from oracle import mepol_oracle as O  # noqa: E402

rng = np.random.default_rng(5)
NT, T, NF = 400, 50, 63
states = rng.standard_normal((NT, T + 1, NF)).astype(np.float32)
X = np.ascontiguousarray(states[:, 1:].reshape(-1, NF))
Xt = torch.as_tensor(X, device="cuda")
Do, Io = O.knn_exact(X, 51)
for split in (0, 4, 16):
    print("plan", ops.knn_plan(len(X), len(X), NF, 51, split), flush=True)
    for rep in range(3):
        D, I, _, nfb = ops.knn(Xt, 51, split=split, return_fallback=True)
        torch.cuda.synchronize()
        Dn, In = D.cpu().numpy(), I.cpu().numpy()
        bad = np.nonzero(~(Dn == Do).all(1) | ~(In == Io).all(1))[0]
        print(f"split {split} rep {rep}: fallback {int(nfb.item())}, rows wrong {len(bad)}",
              bad[:10], flush=True)
