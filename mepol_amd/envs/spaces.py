"""Minimal Box space (the subset of gym.spaces.Box the MEPOL path touches), gym-free."""
import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        if shape is not None and np.isscalar(low):
            low = np.full(shape, low)
            high = np.full(shape, high)
        self.low = np.asarray(low, dtype=self.dtype)
        self.high = np.asarray(high, dtype=self.dtype)
        self.shape = self.low.shape
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def sample(self):
        return self.np_random.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def sample_torch(self, n, device, generator=None):
        """n uniform samples as a float64 tensor on `device` (f32-rounded like sample())."""
        import torch

        lo = torch.as_tensor(self.low, dtype=torch.float64, device=device)
        hi = torch.as_tensor(self.high, dtype=torch.float64, device=device)
        u = torch.rand((n,) + tuple(self.shape), dtype=torch.float64, device=device,
                       generator=generator)
        x = lo + (hi - lo) * u
        return x.to(torch.float32).to(torch.float64) if self.dtype == np.float32 else x

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and np.all(x >= self.low) and np.all(x <= self.high)
