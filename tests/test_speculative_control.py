"""The speculative device-loop protocol (algorithms/device_loop.py: step(speculate), cancel(),
step_start_params()) driven through mepol()'s off-policy loop against the reference's own
decisions, on CPU.

tests/golden/control_*.npz were produced by running the REFERENCE mepol() with scripted
(loss, KL) values (make_golden.py: gen_control).  Here a stand-in for DeviceIteration replays
the same script with the device loop's semantics: a replay applies one update to the target
(+1 on every parameter, as the reference's scripted policy_update), a speculative replay is
launched before the previous one's values are returned, and cancel() undoes a replay the
reference never ran (its update and its script entry).  The CSV rows and the sequence of
(update, lr) / (KL, log_std) the reference recorded must come out unchanged.
"""
import json
import os

import pytest
import torch

from conftest import load_golden
from mepol_amd.algorithms import device_loop
from mepol_amd.algorithms import mepol as M
from mepol_amd.algorithms import particles as P
from mepol_amd.policy import GaussianPolicy

SCENARIOS = ["accept_all", "reject_then_bt", "first_step_rejected", "nan_loss", "no_backtracking",
             "bt_exhausted"]


class _FakeBatch:
    def behavioral_logp(self, policy):
        return torch.zeros(1, dtype=torch.float64)

    def seed_behavioral_logp(self, policy, logp):
        pass


class _FakeLoop:
    """DeviceIteration's host protocol over a scripted sequence of (loss, KL)."""

    tracks_shadow = True

    def __init__(self, state, optimizer, target):
        self.s, self.opt, self.tgt = state, optimizer, target
        self.inflight = []
        self.last = None
        self.logp = torch.zeros(1, dtype=torch.float64)

    def load(self, batch, logp_b=None):
        pass

    def refresh(self):
        pass

    def start_from_behavioral(self):
        return self.logp

    def logp_of_last_step(self):
        # the device loop's contract: nothing in flight and the returned step launched last
        assert not self.inflight and self.last["i"] == self.s["next"] - 1
        self.s["final_logp_reads"] += 1
        return self.logp

    def _launch(self):
        s = self.s
        i = s["next"]
        s["next"] += 1
        s["launched"] += 1
        rec = {"i": i, "lr": self.opt.param_groups[0]["lr"],
               "shadow": [p.detach().clone() for p in self.tgt.parameters()]}
        with torch.no_grad():
            for p in self.tgt.parameters():
                p.add_(1.0)
        loss = float("nan") if i in s["sc"]["nan_loss"] else -1.0 - i
        rec.update(H=-loss, KL=s["sc"]["kls"][i], log_std=float(self.tgt.log_std.detach()[0]))
        self.inflight.append(rec)

    def step(self, speculate=False):
        if not self.inflight:
            self._launch()
        rec = self.inflight.pop(0)
        if speculate and not self.inflight:
            self._launch()
            self.s["speculative"] += 1
        self.last = rec
        self.s["trace"] += [["update", rec["i"], rec["lr"]],
                            ["kl", rec["i"], rec["KL"], rec["log_std"]]]
        return rec["H"], rec["KL"]

    def cancel(self):
        while self.inflight:
            rec = self.inflight.pop()
            self.s["next"] -= 1       # the reference never ran this step
            self.s["cancelled"] += 1
            with torch.no_grad():
                for p, v in zip(self.tgt.parameters(), rec["shadow"]):
                    p.copy_(v)

    def step_start_params(self):
        return self.last["shadow"]


def _strip_time(csv1):
    return [",".join(line.split(",")[:5]) for line in csv1.strip().splitlines()]


@pytest.mark.parametrize("name", SCENARIOS)
def test_speculative_loop_matches_reference_control(name, tmp_path, monkeypatch):
    z = load_golden(f"control_{name}")
    sc = json.loads(str(z["scenario"]))
    state = {"sc": sc, "next": 0, "trace": [], "launched": 0, "speculative": 0, "cancelled": 0,
             "final_logp_reads": 0}

    def fake_collect(env, pol, num_traj, traj_len, state_filter, k, num_workers):
        zz = torch.zeros((num_traj, traj_len + 1, 2), dtype=torch.float64)
        return (zz, zz[:, :-1], torch.full((num_traj, 1), traj_len, dtype=torch.int64), None,
                torch.ones((4, k + 1), dtype=torch.float64), torch.zeros((4, k + 1), dtype=torch.int64))

    monkeypatch.setattr(M, "collect_particles_and_compute_knn", fake_collect)
    monkeypatch.setattr(M, "compute_entropy", lambda *a, **kw: torch.tensor(1.25, dtype=torch.float64))
    monkeypatch.setattr(P, "lookup", lambda *a, **kw: _FakeBatch())
    monkeypatch.setattr(device_loop, "supported", lambda *a, **kw: True)
    monkeypatch.setattr(device_loop, "get",
                        lambda tgt, opt, *a, **kw: _FakeLoop(state, opt, tgt))

    class _Env:
        num_features = 2

        def seed(self, s):
            pass

    M.mepol(env=_Env(), env_name="Scripted", state_filter=None,
            create_policy=lambda is_behavioral=False: GaussianPolicy([4], 2, 2, 0.0), k=4,
            kl_threshold=1.0, max_off_iters=sc["max_off_iters"], use_backtracking=sc["bt"],
            backtrack_coeff=2, max_backtrack_try=4, eps=0.0, learning_rate=0.01, num_traj=2,
            traj_len=3, num_epochs=2, optimizer="adam", full_entropy_traj_scale=1,
            full_entropy_k=4, heatmap_every=1000, heatmap_discretizer=None, heatmap_episodes=1,
            heatmap_num_steps=1, heatmap_cmap=None, heatmap_labels=None, heatmap_interp=None,
            seed=0, out_path=str(tmp_path), num_workers=1)
    csv1 = open(os.path.join(tmp_path, "Scripted.csv")).read()
    csv3 = open(os.path.join(tmp_path, "Scripted_off_policy_iter.csv")).read()
    assert csv3 == str(z["csv3"])
    assert _strip_time(csv1) == _strip_time(str(z["csv1"]))
    assert [list(t) for t in json.loads(str(z["trace"]))] == state["trace"]
    # the protocol was exercised: replays were launched ahead, and every one the reference
    # did not run was cancelled
    assert state["speculative"] > 0
    assert state["launched"] - state["cancelled"] == len(state["trace"]) // 2
    if name in ("reject_then_bt", "first_step_rejected", "no_backtracking"):
        assert state["cancelled"] > 0
