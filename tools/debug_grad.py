"""Per-parameter gradient of one policy_update: GPU eager path vs the oracle's CPU autograd."""
import copy
import os
import sys

import numpy as np
import scipy.special
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle.mepol_oracle as O  # noqa: E402
from mepol_amd import policy as PM  # noqa: E402
from mepol_amd.algorithms import mepol as M  # noqa: E402

NT, T, NF, A, K, HID = 16, 1250, 29, 8, 10, [64, 48]
if len(sys.argv) > 1:
    PM.SPLITK_MIN_ROWS = int(sys.argv[1])
rng = np.random.default_rng(5)
states = rng.standard_normal((NT, T + 1, NF)).astype(np.float32)
actions = (0.5 * rng.standard_normal((NT, T, A))).astype(np.float32)
dev = torch.device("cuda")
st = torch.as_tensor(states, dtype=torch.float64, device=dev)
ac = torch.as_tensor(actions, dtype=torch.float64, device=dev)
rtl = torch.full((NT, 1), T, dtype=torch.int64, device=dev)
nxt = torch.as_tensor(states[:, 1:].reshape(-1, NF), device=dev)
torch.manual_seed(5)
beh = PM.GaussianPolicy(HID, NF, A)
sd = copy.deepcopy(beh.state_dict())
beh = beh.to(dev)
tgt = copy.deepcopy(beh)
opt = torch.optim.SGD(tgt.parameters(), lr=0.0)
s, a, rl, _, D, I = M.make_particle_batch(st, ac, rtl, nxt, K)
G = float(scipy.special.gamma(NF / 2 + 1))
B = float(np.log(K) - scipy.special.digamma(K))
loss, _ = M.policy_update(opt, beh, tgt, s, a, NT, rl, D, I, K, G, B, NF, 0.0)
ob = O.TorchPolicy(HID, NF, A)
ob.load_state_dict(sd)
ot = copy.deepcopy(ob)
oopt = torch.optim.SGD(ot.parameters(), lr=0.0)
oloss, _ = O.torch_policy_update(oopt, ob, ot, torch.as_tensor(states, dtype=torch.float64),
                                 torch.as_tensor(actions, dtype=torch.float64),
                                 NT, rtl.cpu(), D.cpu(), I.cpu(), K, G, B, NF, 0.0)
print("loss gpu", float(loss), "oracle", float(oloss))
gp = dict(tgt.named_parameters())
for n, p in ot.named_parameters():
    g1 = gp[n].grad.cpu().numpy()
    g2 = p.grad.numpy()
    print(f"{n:14s} max|g| {np.abs(g2).max():.3e}  max|diff| {np.abs(g1 - g2).max():.3e}")
