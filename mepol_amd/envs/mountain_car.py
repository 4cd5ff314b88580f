"""Continuous MountainCar with the goal clipped to a wall (never done).

Mirrors src/envs/mountain_car_wall.py:7-45 of the reference and the gym 0.17.2
Continuous_MountainCarEnv constants it inherits (position in [-1.2, 0.6], |v| <= 0.07,
power 0.0015, goal 0.45, reset p ~ U(-0.6, -0.4), v = 0).  The single-env numpy API is kept
for callers that step envs one at a time; the MEPOL rollout steps whole batches on the GPU
(``batched_kind``, csrc/envs.hip).
"""
import math

import numpy as np

from .spaces import Box


class MountainCarContinuous:
    batched_kind = "mountaincar"

    def __init__(self):
        self.min_action = -1.0
        self.max_action = 1.0
        self.min_position = -1.2
        self.max_position = 0.6
        self.max_speed = 0.07
        self.goal_position = 0.45
        self.goal_velocity = 0.0
        self.power = 0.0015
        self.num_features = 2
        self.low_state = np.array([self.min_position, -self.max_speed], dtype=np.float32)
        self.high_state = np.array([self.max_position, self.max_speed], dtype=np.float32)
        self.action_space = Box(self.min_action, self.max_action, shape=(1,), dtype=np.float32)
        self.observation_space = Box(self.low_state, self.high_state, dtype=np.float32)
        self.np_random = np.random.RandomState()
        self.state = None

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def reset(self):
        self.state = np.array([self.np_random.uniform(low=-0.6, high=-0.4), 0.0])
        return np.array(self.state)

    def reset_batch_torch(self, n, device, generator=None):
        """n initial states [n, 2] f64 on device (same distribution as reset())."""
        import torch

        s = torch.zeros((n, 2), dtype=torch.float64, device=device)
        s[:, 0] = -0.6 + 0.2 * torch.rand(n, dtype=torch.float64, device=device, generator=generator)
        return s

    def step(self, action):
        p, v = float(self.state[0]), float(self.state[1])
        force = min(max(action[0], -1.0), 1.0)
        v += force * self.power - 0.0025 * math.cos(3 * p)
        v = min(max(v, -self.max_speed), self.max_speed)
        p += v
        p = min(max(p, self.min_position), self.max_position)
        if p == self.min_position and v < 0:
            v = 0
        if p > self.goal_position:
            p = self.goal_position
            v = 0.0
        self.state = np.array([p, v])
        reward = -math.pow(action[0], 2) * 0.1
        return self.state, reward, False, {}
