from . import VecEnv, VecEnvWrapper, CloudpickleWrapper, clear_mpi_env_vars  # noqa: F401
