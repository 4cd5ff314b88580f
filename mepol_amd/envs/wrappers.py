"""ErgodicEnv: ignore the done signal (src/envs/wrappers.py:4-15)."""


class ErgodicEnv:
    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    @property
    def unwrapped(self):
        e = self.env
        while isinstance(e, ErgodicEnv):
            e = e.env
        return e

    def reset(self):
        return self.env.reset()

    def seed(self, seed=None):
        return self.env.seed(seed)

    def step(self, a):
        s, r, _, i = self.env.step(a)
        return s, r, False, i


def unwrap(env):
    while hasattr(env, "env") and not hasattr(type(env), "batched_kind"):
        env = env.env
    return env
