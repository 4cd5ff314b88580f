"""Continuous 2-D GridWorld with walls (src/envs/gridworld_continuous.py:34-154, walls :66-76).

Single-env numpy API for compatibility; the MEPOL rollout steps batches on the GPU
(``batched_kind``, csrc/envs.hip).  Rendering (pygame) is out of scope.
"""
import numpy as np

from .spaces import Box


class GridWorldContinuous:
    batched_kind = "gridworld"

    def __init__(self, dim=6, max_delta=0.2, wall_width=2.5):
        self.num_features = 2
        self.dim = dim
        self.max_delta = max_delta
        self.wall_width = wall_width
        ma = np.array([max_delta, max_delta], dtype=np.float32)
        self.action_space = Box(-ma, ma, dtype=np.float32)
        mp = np.array([dim, dim], dtype=np.float32)
        self.observation_space = Box(-mp, mp, dtype=np.float32)
        self.init_states = Box(np.array([-dim, -dim], dtype=np.float32),
                               np.array([-dim + 2, -dim + 2], dtype=np.float32), dtype=np.float32)
        h, w, d = wall_width / 2, wall_width, dim
        # (xmin, xmax, ymin, ymax), closed boxes
        self.walls = [(-h, h, -w, w), (-w, -h, -h, h), (h, w, -h, h), (-d, -(d - w), -h, h),
                      (-h, h, -d, -(d - w)), (d - w, d, -h, h), (-h, h, d - w, d)]
        self.state = None

    def seed(self, seed=None):
        self.init_states.seed(seed)
        return [seed]

    def reset(self):
        self.state = self.init_states.sample()
        return self.state

    def reset_batch_torch(self, n, device, generator=None):
        """n initial states [n, 2] as f32 tensor on device (same distribution as reset())."""
        return self.init_states.sample_torch(n, device, generator).to(dtype=__import__("torch").float32)

    def step(self, action):
        x, y = self.state
        dx = np.clip(action[0], -self.max_delta, self.max_delta)
        dy = np.clip(action[1], -self.max_delta, self.max_delta)
        nx, ny = float(x) + float(dx), float(y) + float(dy)
        for (x0, x1, y0, y1) in self.walls:
            if x0 <= nx <= x1 and y0 <= ny <= y1:
                nx, ny = x, y
        if abs(nx) >= self.dim or abs(ny) >= self.dim:
            nx, ny = x, y
        self.state = np.array([nx, ny], dtype=np.float32)
        return self.state, 0, False, {}
