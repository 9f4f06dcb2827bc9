"""Minimal gym stand-in (import-time names used by the reference's CrowdSim)."""
from . import spaces  # noqa: F401
from . import envs  # noqa: F401


class Env(object):
    metadata = {}

    def seed(self, seed=None):  # gym.Env.seed default: no-op
        return

    def close(self):
        return

    @property
    def unwrapped(self):
        return self


class Wrapper(Env):
    def __init__(self, env):
        self.env = env


class ObservationWrapper(Wrapper):
    pass


def make(env_id):
    return envs.registration.make(env_id)
