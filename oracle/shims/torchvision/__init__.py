"""torchvision stand-in: convgru_model.py imports it at module level; the srnn path never uses it."""
from . import transforms  # noqa: F401
