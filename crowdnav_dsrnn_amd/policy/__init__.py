"""DSRNN policy (reference: pytorchBaselines/a2c_ppo_acktr/{model,srnn_model,distributions}.py)."""
from .convgru_model import ConvGRU  # noqa: F401
from .model import Policy  # noqa: F401
from .srnn_model import SRNN  # noqa: F401
