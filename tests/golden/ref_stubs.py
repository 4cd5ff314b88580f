"""Import shims that let the read-only reference (/root/reference) run in this container.

Test infrastructure only (used by ``make_golden.py``; never imported by the product or on
the GPU box).  The reference needs three packages that are not installed here
(SURVEY.md §8c):

* ``gym`` 0.17.2 -- only ``Env``, ``Wrapper``, ``spaces.Box`` and the
  ``Continuous_MountainCarEnv`` base class are touched by the MEPOL path.  The base-class
  constants below are gym 0.17.2's published values (min/max position -1.2/0.6, max speed
  0.07, goal 0.45, power 0.0015, reset p ~ U(-0.6, -0.4), v = 0).  They cannot be verified
  offline; the dynamics themselves live in the reference's own ``step``
  (``src/envs/mountain_car_wall.py:13-45``).
* ``pygame`` -- render only (``src/envs/gridworld_continuous.py:8``).
* ``torch.utils.tensorboard`` -- ``SummaryWriter`` used for logging
  (``src/algorithms/mepol.py:14``); replaced by a no-op writer.
"""
import sys
import types

import numpy as np


def _make_gym():
    gym = types.ModuleType("gym")

    class Env:
        def seed(self, seed=None):
            self.np_random = np.random.RandomState(seed)
            return [seed]

    class Wrapper(Env):
        def __init__(self, env):
            self.env = env
            self.action_space = env.action_space
            self.observation_space = env.observation_space

        def __getattr__(self, name):
            if name.startswith("_") or name == "env":
                raise AttributeError(name)
            return getattr(self.env, name)

        def reset(self, **kw):
            return self.env.reset(**kw)

        def step(self, a):
            return self.env.step(a)

        def seed(self, seed=None):
            return self.env.seed(seed)

    class Box:
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.dtype = np.dtype(dtype)
            if shape is not None and np.isscalar(low):
                low = np.full(shape, low, dtype=self.dtype)
                high = np.full(shape, high, dtype=self.dtype)
            self.low = np.asarray(low, dtype=self.dtype)
            self.high = np.asarray(high, dtype=self.dtype)
            self.shape = self.low.shape
            self.np_random = np.random.RandomState()

        def seed(self, seed=None):
            self.np_random = np.random.RandomState(seed)

        def sample(self):
            return self.np_random.uniform(self.low, self.high, self.shape).astype(self.dtype)

    spaces = types.ModuleType("gym.spaces")
    spaces.Box = Box

    class Continuous_MountainCarEnv(Env):
        def __init__(self):
            self.min_action = -1.0
            self.max_action = 1.0
            self.min_position = -1.2
            self.max_position = 0.6
            self.max_speed = 0.07
            self.goal_position = 0.45
            self.goal_velocity = 0.0
            self.power = 0.0015
            self.low_state = np.array([self.min_position, -self.max_speed], dtype=np.float32)
            self.high_state = np.array([self.max_position, self.max_speed], dtype=np.float32)
            self.action_space = Box(self.min_action, self.max_action, shape=(1,), dtype=np.float32)
            self.observation_space = Box(self.low_state, self.high_state, dtype=np.float32)
            self.seed()
            self.state = None

        def reset(self):
            self.state = np.array([self.np_random.uniform(low=-0.6, high=-0.4), 0])
            return np.array(self.state)

    envs = types.ModuleType("gym.envs")
    cc = types.ModuleType("gym.envs.classic_control")
    cmc = types.ModuleType("gym.envs.classic_control.continuous_mountain_car")
    cmc.Continuous_MountainCarEnv = Continuous_MountainCarEnv

    gym.Env = Env
    gym.Wrapper = Wrapper
    gym.spaces = spaces
    gym.envs = envs
    envs.classic_control = cc
    cc.continuous_mountain_car = cmc
    return {
        "gym": gym,
        "gym.spaces": spaces,
        "gym.envs": envs,
        "gym.envs.classic_control": cc,
        "gym.envs.classic_control.continuous_mountain_car": cmc,
    }


def install(reference_root="/root/reference"):
    """Register the shims in ``sys.modules`` and put the reference on ``sys.path``."""
    for name, mod in _make_gym().items():
        sys.modules.setdefault(name, mod)
    sys.modules.setdefault("pygame", types.ModuleType("pygame"))

    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        def __init__(self, *a, **kw):
            pass

        def add_scalar(self, *a, **kw):
            pass

        def add_figure(self, *a, **kw):
            pass

    tb.SummaryWriter = SummaryWriter
    import torch.utils

    sys.modules["torch.utils.tensorboard"] = tb
    torch.utils.tensorboard = tb
    if reference_root not in sys.path:
        sys.path.insert(0, reference_root)
