"""Policy wrapper (pytorchBaselines/a2c_ppo_acktr/model.py:17-104): base='srnn' or 'convgru' + DiagGaussian.

API and return values as in the reference:
  act(inputs, rnn_hxs, masks, deterministic=False) -> value (E,1), action (E,2), log_prob (E,1), rnn_hxs
  get_value(inputs, rnn_hxs, masks) -> value (E,1)
  evaluate_actions(inputs, rnn_hxs, masks, action) -> value, log_prob, entropy, rnn_hxs
`base.nenv` is writable (test.py:199) and `base.human_num` readable (evaluation.py:34).
"""
import torch
import torch.nn as nn

from .. import ops
from .convgru_model import ConvGRU
from .distributions import DiagGaussian
from .srnn_model import SRNN


class Policy(nn.Module):
    def __init__(self, obs_shape, action_space, base=None, base_kwargs=None):
        super().__init__()
        if base == "srnn":
            self.base = SRNN(obs_shape, base_kwargs)
            self.srnn, self.convgru = True, False
            dist_in = self.base.output_size
        elif base == "convgru":   # model.py:25-33: the LiDAR policy; its distribution reads actor.fc2 (64)
            self.base = ConvGRU(obs_shape, base_kwargs)
            self.srnn, self.convgru = False, True
            dist_in = self.base.actor.fc2.out_features
        else:
            raise NotImplementedError("base must be 'srnn' or 'convgru'")
        if action_space.__class__.__name__ != "Box":
            raise NotImplementedError("CrowdSimDict drives a Box(2,) action space")
        self.dist = DiagGaussian(dist_in, action_space.shape[0])

    @property
    def is_recurrent(self):
        return self.base.is_recurrent

    def forward(self, inputs, rnn_hxs, masks):
        raise NotImplementedError

    def _infer(self, inputs, rnn_hxs, masks, out_hxs=None):
        if self.srnn:
            return self.base(inputs, rnn_hxs, masks, infer=True, out_hxs=out_hxs)
        return self.base(inputs, rnn_hxs, masks)

    def act(self, inputs, rnn_hxs, masks, deterministic=False, out_hxs=None):
        """out_hxs (optional, srnn, no-grad): tensors that receive the new recurrent state (SRNN.forward)."""
        value, actor_features, rnn_hxs = self._infer(inputs, rnn_hxs, masks, out_hxs)
        if actor_features.is_cuda and not torch.is_grad_enabled() and isinstance(self.dist, DiagGaussian):
            # sample / mode and log_probs of the same distribution in one launch (ops.gaussian_act)
            d = self.dist
            action, action_log_probs = ops.gaussian_act(d.fc_mean(actor_features), d.logstd._bias.view(-1),
                                                        deterministic)
            return value, action, action_log_probs, rnn_hxs
        dist = self.dist(actor_features)
        action = dist.mode() if deterministic else dist.sample()
        action_log_probs = dist.log_probs(action)
        return value, action, action_log_probs, rnn_hxs

    def get_value(self, inputs, rnn_hxs, masks):
        value, _, _ = self._infer(inputs, rnn_hxs, masks)
        return value

    def evaluate_actions(self, inputs, rnn_hxs, masks, action):
        value, actor_features, rnn_hxs = self.base(inputs, rnn_hxs, masks)
        dist = self.dist(actor_features)
        action_log_probs = dist.log_probs(action)
        dist_entropy = dist.entropy().mean()
        return value, action_log_probs, dist_entropy, rnn_hxs
