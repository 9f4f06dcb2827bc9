"""Policy wrapper (pytorchBaselines/a2c_ppo_acktr/model.py:17-104): base='srnn' + DiagGaussian.

API and return values as in the reference:
  act(inputs, rnn_hxs, masks, deterministic=False) -> value (E,1), action (E,2), log_prob (E,1), rnn_hxs
  get_value(inputs, rnn_hxs, masks) -> value (E,1)
  evaluate_actions(inputs, rnn_hxs, masks, action) -> value, log_prob, entropy, rnn_hxs
`base.nenv` is writable (test.py:199) and `base.human_num` readable (evaluation.py:34).
"""
import torch.nn as nn

from .distributions import DiagGaussian
from .srnn_model import SRNN


class Policy(nn.Module):
    def __init__(self, obs_shape, action_space, base=None, base_kwargs=None):
        super().__init__()
        if base != "srnn":
            raise NotImplementedError("only base='srnn' is provided (the ConvGRU/LiDAR policy is out of scope)")
        self.base = SRNN(obs_shape, base_kwargs)
        self.srnn = True
        if action_space.__class__.__name__ != "Box":
            raise NotImplementedError("DSRNN drives a Box(2,) action space")
        self.dist = DiagGaussian(self.base.output_size, action_space.shape[0])

    @property
    def is_recurrent(self):
        return self.base.is_recurrent

    def forward(self, inputs, rnn_hxs, masks):
        raise NotImplementedError

    def act(self, inputs, rnn_hxs, masks, deterministic=False):
        value, actor_features, rnn_hxs = self.base(inputs, rnn_hxs, masks, infer=True)
        dist = self.dist(actor_features)
        action = dist.mode() if deterministic else dist.sample()
        action_log_probs = dist.log_probs(action)
        return value, action, action_log_probs, rnn_hxs

    def get_value(self, inputs, rnn_hxs, masks):
        value, _, _ = self.base(inputs, rnn_hxs, masks, infer=True)
        return value

    def evaluate_actions(self, inputs, rnn_hxs, masks, action):
        value, actor_features, rnn_hxs = self.base(inputs, rnn_hxs, masks)
        dist = self.dist(actor_features)
        action_log_probs = dist.log_probs(action)
        dist_entropy = dist.entropy().mean()
        return value, action_log_probs, dist_entropy, rnn_hxs
