"""Small helpers mirrored from pytorchBaselines/a2c_ppo_acktr/utils.py:32-56."""
import torch.nn as nn


class AddBias(nn.Module):
    """utils.py:32-43 — a learnable bias stored as a column (state_dict key `_bias`, shape (n, 1))."""

    def __init__(self, bias):
        super().__init__()
        self._bias = nn.Parameter(bias.unsqueeze(1))

    def forward(self, x):
        if x.dim() == 2:
            bias = self._bias.t().view(1, -1)
        else:
            bias = self._bias.t().view(1, -1, 1, 1)
        return x + bias


def init(module, weight_init, bias_init, gain=1):
    """utils.py:53-56."""
    weight_init(module.weight.data, gain=gain)
    bias_init(module.bias.data)
    return module


def update_linear_schedule(optimizer, epoch, total_num_epochs, initial_lr):
    """utils.py:46-50."""
    lr = initial_lr - (initial_lr * (epoch / float(total_num_epochs)))
    for param_group in optimizer.param_groups:
        param_group["lr"] = lr


class Linear(nn.Linear):
    """nn.Linear (same parameters and state_dict keys) whose training backward uses a split-K weight
    gradient (ops.linear): these layers see T*B or T*B*N rows in PPO minibatches."""

    def forward(self, x):
        from .. import ops

        return ops.linear(x, self.weight, self.bias)
