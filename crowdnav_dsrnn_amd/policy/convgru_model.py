"""ConvGRU policy base for the LiDAR observation (pytorchBaselines/a2c_ppo_acktr/convgru_model.py:21-211).

Same module tree and state_dict keys as the reference (conv_blk.conv1..3, gru, actor.fc1/fc2,
critic.fc1/fc2, critic_linear): Conv1d(1,512,7,2) -> Conv1d(512,256,5,2) -> Conv1d(256,128,3,2), each with
LeakyReLU, then [MaxPool1d(21), AvgPool1d(21)] -> 256 features -> GRU(256, 256) -> actor (256-64-64) /
critic (256-256-256 -> 1). The convolutions are library (MIOpen) calls; the GRU is the mask-segmented GRU
of the DSRNN (ops.masked_gru: HIP gate kernels + GEMMs), whose per-step masking equals the reference's
segmentation at episode starts (convgru_model.py:48-101).

One deliberate difference: the reference squeezes every size-1 dim after pooling (`x.squeeze()`,
convgru_model.py:203), which also drops the batch dim when it is 1 and then fails in _forward_gru (test.py
evaluates with one env); only the pooled length dim is squeezed here.
"""
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .utils import Linear, init


class ConvGRU(nn.Module):
    def __init__(self, obs_space, config):
        super().__init__()
        self.config = config
        self._init_ = lambda m: init(m, nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0), np.sqrt(2))
        self.actor_hidden_size = 64
        self.critic_hidden_size = 256
        self.gru_input_size = 256
        self.shared_ac_size = 256
        self._hidden_size = self.shared_ac_size
        self._recurrent = True
        self.gru = nn.GRU(self.gru_input_size, self.shared_ac_size)
        for name, param in self.gru.named_parameters():
            if "bias" in name:
                nn.init.constant_(param, 0)
            elif "weight" in name:
                nn.init.orthogonal_(param)
        self.conv_blk = nn.Sequential(OrderedDict([
            ("conv1", self._init_(nn.Conv1d(1, 512, 7, 2))), ("lrelu1", nn.LeakyReLU()),
            ("conv2", self._init_(nn.Conv1d(512, 256, 5, 2))), ("lrelu2", nn.LeakyReLU()),
            ("conv3", self._init_(nn.Conv1d(256, 128, 3, 2))), ("lrelu3", nn.LeakyReLU()),
        ]))
        self.ap = nn.AvgPool1d(kernel_size=21, stride=1, padding=0)
        self.mp = nn.MaxPool1d(kernel_size=21, stride=1, padding=0)
        self.actor = nn.Sequential(OrderedDict([
            ("fc1", self._init_(Linear(self.shared_ac_size, self.actor_hidden_size))), ("tanh1", nn.Tanh()),
            ("fc2", self._init_(Linear(self.actor_hidden_size, self.actor_hidden_size))), ("tanh2", nn.Tanh()),
        ]))
        self.critic = nn.Sequential(OrderedDict([
            ("fc1", self._init_(Linear(self.shared_ac_size, self.critic_hidden_size))), ("tanh1", nn.Tanh()),
            ("fc2", self._init_(Linear(self.critic_hidden_size, self.critic_hidden_size))), ("tanh2", nn.Tanh()),
        ]))
        self.critic_linear = self._init_(Linear(self.critic_hidden_size, 1))
        self.train()

    @property
    def is_recurrent(self):
        return self._recurrent

    @property
    def recurrent_hidden_state_size(self):
        return self._hidden_size

    @property
    def output_size(self):
        return self._hidden_size

    def _forward_gru(self, x, hxs, masks):
        """convgru_model.py:48-101: one step when x has as many rows as hxs, else a (T*N) sequence."""
        g = self.gru
        w = (g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0)
        N = hxs.size(0)
        T = x.size(0) // N
        out, h = ops.masked_gru(x.view(T, N, x.size(1)), hxs, masks.reshape(T, N), *w)
        return out.reshape(T * N, -1), h

    def forward(self, inputs, rnn_hxs, masks):
        x = self.conv_blk(inputs)
        x = torch.cat([self.mp(x), self.ap(x)], dim=1).squeeze(-1)
        x, rnn_hxs = self._forward_gru(x, rnn_hxs, masks)
        return self.critic_linear(self.critic(x)), self.actor(x), rnn_hxs
