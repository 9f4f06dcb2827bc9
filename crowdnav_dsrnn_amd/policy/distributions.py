"""Action distribution of the Box action space (pytorchBaselines/a2c_ppo_acktr/distributions.py:36-94)."""
import torch
import torch.nn as nn

from .utils import AddBias, Linear, init


class FixedNormal(torch.distributions.Normal):
    """distributions.py:36-45: log_probs summed over action dims, mode = mean.

    Built with validate_args=False: torch's default argument validation reduces loc / scale / the
    actions to a host bool (three device->host synchronisations per act()); it only raises on NaN or
    non-positive inputs and never changes a value."""

    def __init__(self, loc, scale):
        super().__init__(loc, scale, validate_args=False)

    def sample(self, sample_shape=torch.Size()):
        """loc + scale * N(0, 1): the draw torch.normal(loc, scale) makes, without its std >= 0 check
        (a device min + host read per call)."""
        shape = self._extended_shape(sample_shape)
        with torch.no_grad():
            eps = torch.randn(shape, dtype=self.loc.dtype, device=self.loc.device)
            return eps * self.scale.expand(shape) + self.loc.expand(shape)

    def log_probs(self, actions):
        return super().log_prob(actions).sum(-1, keepdim=True)

    def entrop(self):
        return super().entropy().sum(-1)

    def mode(self):
        return self.mean


class DiagGaussian(nn.Module):
    """distributions.py:74-94: mean from a linear layer, state-independent log-std (AddBias on zeros)."""

    def __init__(self, num_inputs, num_outputs):
        super().__init__()
        self.fc_mean = init(Linear(num_inputs, num_outputs), nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0))
        self.logstd = AddBias(torch.zeros(num_outputs))

    def forward(self, x):
        action_mean = self.fc_mean(x)
        action_logstd = self.logstd(torch.zeros_like(action_mean))
        return FixedNormal(action_mean, action_logstd.exp())
