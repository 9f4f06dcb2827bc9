from . import VecEnvWrapper


class VecNormalize(VecEnvWrapper):
    pass
