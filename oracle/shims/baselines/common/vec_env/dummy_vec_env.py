from . import VecEnv


class DummyVecEnv(VecEnv):
    pass
