"""OpenAI-baselines stand-in: import-time names used by the reference's envs.py / shmem_vec_env.py.
Only class/func names are provided; the fixture generator drives CrowdSimDict directly and
restates the VecEnv auto-reset + Monitor bookkeeping itself (oracle/gen_golden.py)."""
from . import bench  # noqa: F401
