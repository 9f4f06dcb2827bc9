import contextlib


class VecEnv(object):
    def __init__(self, num_envs, observation_space, action_space):
        self.num_envs = num_envs
        self.observation_space = observation_space
        self.action_space = action_space


class VecEnvWrapper(VecEnv):
    def __init__(self, venv, observation_space=None, action_space=None):
        self.venv = venv
        VecEnv.__init__(self, venv.num_envs, observation_space or venv.observation_space,
                        action_space or venv.action_space)


class CloudpickleWrapper(object):
    def __init__(self, x):
        self.x = x


@contextlib.contextmanager
def clear_mpi_env_vars():
    yield
