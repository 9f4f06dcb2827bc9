"""On-device PPO learner for the DSRNN policy.

Same classes and methods as the reference's pytorchBaselines/a2c_ppo_acktr/{storage.py,algo/ppo.py}, kept
resident on the GPU; with torch.distributed initialised (one process per GPU, backend "nccl" = RCCL)
the gradients are all-reduced per minibatch and the advantage normalisation uses global statistics.
"""
from .ppo import PPO  # noqa: F401
from .storage import RolloutStorage, SRNNRolloutStorage  # noqa: F401
