"""DSRNN (structural-RNN) actor-critic for the crowd-navigation observation dict.

Same module tree, parameter names and initialisation as the reference
(pytorchBaselines/a2c_ppo_acktr/srnn_model.py:9-504), so `state_dict()` keys match the reference
checkpoints (data/example_model*/checkpoints/*.pt) one to one. The compute is organised for the GPU:

  * the three input layers — HumanHumanEdgeRNN.encoder_linear + ReLU for the temporal and spatial
    edges (srnn_model.py:210-211), SRNN.robot_linear (:466) and HumanNodeRNN.encoder_linear + ReLU
    (:160-161) — run as ONE fused HIP kernel (`crowdnav_dsrnn_amd.ops.edge_features`) over every env
    (and time step) instead of four small GEMM launches;
  * the GRUs keep torch.nn.GRU's parameters but run as the native mask-segmented sequence kernels
    (`ops.masked_gru` / `ops.masked_gru_group`; the spatial and temporal edge RNNs share launches): the
    recurrent masks are applied per step on the device (no host synchronisation), which equals the
    reference's any-zero segmentation (srnn_model.py:52-104): inside a segment every mask is 1;
  * the spatial-edge attention is batched over envs, humans and time steps.
"""
import numpy as np
import torch
import torch.nn as nn

from .. import ops
from .utils import Linear, init


class RNNBase(nn.Module):
    """GRU holder (srnn_model.py:9-32): orthogonal weights, zero biases."""

    def __init__(self, config, edge):
        super().__init__()
        self.config = config
        if edge:
            self.gru = nn.GRU(config.SRNN.human_human_edge_embedding_size, config.SRNN.human_human_edge_rnn_size)
        else:
            self.gru = nn.GRU(config.SRNN.human_node_embedding_size * 2, config.SRNN.human_node_rnn_size)
        for name, param in self.gru.named_parameters():
            if "bias" in name:
                nn.init.constant_(param, 0)
            elif "weight" in name:
                nn.init.orthogonal_(param)

    def masked_gru(self, x, h0, masks):
        """x (T, B, F), h0 (B, H), masks (T, B) -> out (T, B, H), h_T (B, H).
        h <- h * mask[t] before step t (episode starts), then one GRU step (srnn_model.py:52-104);
        runs as ops.masked_gru (HIP gate kernels + GEMMs)."""
        g = self.gru
        return ops.masked_gru(x, h0, masks, g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0)

    def infer_step(self, x, h0, m, dest):
        """T = 1 without autograd: ops.gru_infer_step (new state also written into `dest`, which may be a
        slice of the (B, N + 1, H) state tensor and may alias h0)."""
        g = self.gru
        if x.is_cuda and g.weight_hh_l0.shape[1] % 32 == 0:   # input projection in the step kernel
            return ops.gru_infer_group((x, h0, m, g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0,
                                        dest))[0]
        return ops.gru_infer_step(x, h0, m, g.weight_ih_l0, g.weight_hh_l0, g.bias_ih_l0, g.bias_hh_l0, dest)


class HumanNodeRNN(RNNBase):
    """Robot node RNN (srnn_model.py:109-173)."""

    def __init__(self, config):
        super().__init__(config, edge=False)
        self.rnn_size = config.SRNN.human_node_rnn_size
        self.output_size = config.SRNN.human_node_output_size
        self.embedding_size = config.SRNN.human_node_embedding_size
        self.input_size = config.SRNN.human_node_input_size
        self.edge_rnn_size = config.SRNN.human_human_edge_rnn_size
        self.encoder_linear = nn.Linear(self.input_size, self.embedding_size)
        self.relu = nn.ReLU()
        self.edge_embed = nn.Linear(self.edge_rnn_size, self.embedding_size)  # unused by forward (kept for keys)
        self.edge_attention_embed = Linear(self.edge_rnn_size * 2, self.embedding_size)
        self.output_linear = Linear(self.rnn_size, self.output_size)

    def forward(self, node_embed, h_temporal, h_spatial_other, h, masks, dest=None):
        """node_embed (T,B,64) = relu(encoder_linear(robot_linear(robot_node))) from the fused kernel.
        dest (B, 1, H) selects the no-autograd T = 1 path (the new state is written there)."""
        h_edges = torch.cat((h_temporal, h_spatial_other), -1)
        h_edges_embedded = self.relu(self.edge_attention_embed(h_edges))
        x = torch.cat((node_embed, h_edges_embedded), -1)
        if dest is not None:
            x = self.infer_step(x.reshape(-1, x.shape[-1]), h, masks.reshape(-1), dest)
            return self.output_linear(x.unsqueeze(0)), dest
        x, h_new = self.masked_gru(x, h, masks)
        return self.output_linear(x), h_new


class HumanHumanEdgeRNN(RNNBase):
    """Edge RNN (srnn_model.py:176-215); its encoder_linear+ReLU runs inside the fused kernel."""

    def __init__(self, config):
        super().__init__(config, edge=True)
        self.rnn_size = config.SRNN.human_human_edge_rnn_size
        self.embedding_size = config.SRNN.human_human_edge_embedding_size
        self.input_size = config.SRNN.human_human_edge_input_size
        self.encoder_linear = nn.Linear(self.input_size, self.embedding_size)
        self.relu = nn.ReLU()

    def forward(self, embedded, h, masks):
        return self.masked_gru(embedded, h, masks)


class EdgeAttention(nn.Module):
    """Temporal-vs-spatial edge attention (srnn_model.py:218-339), one head."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.human_human_edge_rnn_size = config.SRNN.human_human_edge_rnn_size
        self.human_node_rnn_size = config.SRNN.human_node_rnn_size
        self.attention_size = config.SRNN.attention_size
        self.temporal_edge_layer = nn.ModuleList([Linear(self.human_human_edge_rnn_size, self.attention_size)])
        self.spatial_edge_layer = nn.ModuleList([Linear(self.human_human_edge_rnn_size, self.attention_size)])
        self.agent_num = 1
        self.num_attention_head = 1

    def forward(self, h_temporal, h_spatials):
        """h_temporal (T,B,256), h_spatials (T,B,N,256) -> weighted (T,B,256), attn (T*B,N,1)."""
        T, B, N, H = h_spatials.shape
        temporal_embed = self.temporal_edge_layer[0](h_temporal)          # (T,B,64)
        scale = N / np.sqrt(self.attention_size)                          # temperature = num_edges / sqrt(d)
        if h_spatials.is_cuda and H in (64, 128, 256) and N <= 64:
            # spatial_edge_layer, scores, softmax and pooling in one pass over h_spatials (ops.spatial_attention)
            sl = self.spatial_edge_layer[0]
            weighted, attn = ops.spatial_attention(h_spatials.reshape(T * B, N, H), temporal_embed.reshape(T * B, -1),
                                                   sl.weight, sl.bias, scale)
            return weighted.reshape(T, B, H), attn
        spatial_embed = self.spatial_edge_layer[0](h_spatials)            # (T,B,N,64)
        attn = (spatial_embed * temporal_embed.unsqueeze(2)).sum(-1)      # (T,B,N)
        attn = attn * scale
        attn = torch.softmax(attn, dim=-1).reshape(T * B, N, 1)
        weighted = ops.attention_pool(h_spatials.reshape(T * B, N, H), attn)  # bmm(hs^T, attn): (T*B, H)
        return weighted.reshape(T, B, H), attn


class SRNN(nn.Module):
    """srnn_model.py:342-504."""

    def __init__(self, obs_space_dict, config, infer=False):
        super().__init__()
        self.infer = infer
        self.is_recurrent = True
        self.config = config
        self.human_num = config.sim.human_num
        self.seq_length = config.ppo.num_steps
        self.nenv = config.training.num_processes
        self.nminibatch = config.ppo.num_mini_batch
        self.human_node_rnn_size = config.SRNN.human_node_rnn_size
        self.human_human_edge_rnn_size = config.SRNN.human_human_edge_rnn_size
        self.output_size = config.SRNN.human_node_output_size

        self.humanNodeRNN = HumanNodeRNN(config)
        self.humanhumanEdgeRNN_spatial = HumanHumanEdgeRNN(config)
        self.humanhumanEdgeRNN_temporal = HumanHumanEdgeRNN(config)
        self.attn = EdgeAttention(config)

        def init_(m):
            return init(m, nn.init.orthogonal_, lambda x: nn.init.constant_(x, 0), np.sqrt(2))

        num_inputs = hidden_size = self.output_size
        self.actor = nn.Sequential(init_(Linear(num_inputs, hidden_size)), nn.Tanh(),
                                   init_(Linear(hidden_size, hidden_size)), nn.Tanh())
        self.critic = nn.Sequential(init_(Linear(num_inputs, hidden_size)), nn.Tanh(),
                                    init_(Linear(hidden_size, hidden_size)), nn.Tanh())
        self.critic_linear = init_(Linear(hidden_size, 1))
        self.robot_linear = init_(nn.Linear(7, 3))
        self.human_node_final_linear = init_(nn.Linear(self.output_size, 2))  # unused by forward (keys)
        self.num_edges = self.human_num + 1

    def forward(self, inputs, rnn_hxs, masks, infer=False, out_hxs=None):
        """srnn_model.py:409-504. `out_hxs` (optional, inference only): preallocated
        {'human_node_rnn': (B,1,128), 'human_human_edge_rnn': (B,N+1,256)} that receive the new state (they
        may be the very tensors of rnn_hxs: the state is updated in place); rnn_hxs then holds them."""
        if infer and not torch.is_grad_enabled():
            return self._infer_step(inputs, rnn_hxs, masks, out_hxs)
        if infer:
            T, B = 1, self.nenv
        else:
            T, B = self.seq_length, self.nenv // self.nminibatch
        N = inputs["spatial_edges"].shape[-2]
        te, se, ne = ops.edge_features(
            inputs["robot_node"].reshape(T * B, 1, 7), inputs["temporal_edges"].reshape(T * B, 1, 2),
            inputs["spatial_edges"].reshape(T * B, N, 2),
            self.humanhumanEdgeRNN_temporal.encoder_linear.weight, self.humanhumanEdgeRNN_temporal.encoder_linear.bias,
            self.humanhumanEdgeRNN_spatial.encoder_linear.weight, self.humanhumanEdgeRNN_spatial.encoder_linear.bias,
            self.robot_linear.weight, self.robot_linear.bias,
            self.humanNodeRNN.encoder_linear.weight, self.humanNodeRNN.encoder_linear.bias)
        m = masks.reshape(T, B)
        h_edge = rnn_hxs["human_human_edge_rnn"].reshape(B, self.num_edges, -1)
        h_node = rnn_hxs["human_node_rnn"].reshape(B, -1)
        H = h_edge.shape[-1]

        # the temporal and spatial edge RNNs are independent and have the same sizes: their rows (B and B*N per
        # step) share every step's launch (ops.masked_gru_group; the temporal RNN alone cannot fill the GPU)
        m_s = m.unsqueeze(-1).expand(T, B, N).reshape(T, B * N)
        x_s, h0_s = se.reshape(T, B * N, 64), h_edge[:, 1:, :].reshape(B * N, H)
        x_t, h0_t = te.reshape(T, B, 64), h_edge[:, 0, :]
        if te.is_cuda and H % 32 == 0:
            gs, gt = self.humanhumanEdgeRNN_spatial.gru, self.humanhumanEdgeRNN_temporal.gru
            (out_s, h_s), (out_t, h_t) = ops.masked_gru_group(
                (x_s, h0_s, m_s, gs.weight_ih_l0, gs.weight_hh_l0, gs.bias_ih_l0, gs.bias_hh_l0),
                (x_t, h0_t, m, gt.weight_ih_l0, gt.weight_hh_l0, gt.bias_ih_l0, gt.bias_hh_l0))
        else:
            out_t, h_t = self.humanhumanEdgeRNN_temporal(x_t, h0_t, m)
            out_s, h_s = self.humanhumanEdgeRNN_spatial(x_s, h0_s, m_s)
        out_s = out_s.reshape(T, B, N, H)
        weighted, _ = self.attn(out_t, out_s)
        outputs, h_n = self.humanNodeRNN(ne.reshape(T, B, 64), out_t, weighted, h_node, m)

        rnn_hxs["human_node_rnn"] = h_n.reshape(B, 1, -1)
        rnn_hxs["human_human_edge_rnn"] = torch.cat((h_t.unsqueeze(1), h_s.reshape(B, N, H)), 1)
        hidden_critic = self.critic(outputs)
        hidden_actor = self.actor(outputs)
        if infer:
            return self.critic_linear(hidden_critic).squeeze(0), hidden_actor.squeeze(0), rnn_hxs
        return self.critic_linear(hidden_critic).view(-1, 1), hidden_actor.view(-1, self.output_size), rnn_hxs

    def _infer_step(self, inputs, rnn_hxs, masks, out_hxs):
        """The act() step without autograd: same arithmetic as the T = 1 path of forward(), but the GRUs
        read the (B, N + 1, H) edge state through strided views and write the new state straight into its
        destination (cn_gru_fwd_step_scatter) instead of slicing copies, a clone and a torch.cat."""
        B = self.nenv
        N = inputs["spatial_edges"].shape[-2]
        te, se, ne = ops.edge_features(
            inputs["robot_node"].reshape(B, 1, 7), inputs["temporal_edges"].reshape(B, 1, 2),
            inputs["spatial_edges"].reshape(B, N, 2),
            self.humanhumanEdgeRNN_temporal.encoder_linear.weight, self.humanhumanEdgeRNN_temporal.encoder_linear.bias,
            self.humanhumanEdgeRNN_spatial.encoder_linear.weight, self.humanhumanEdgeRNN_spatial.encoder_linear.bias,
            self.robot_linear.weight, self.robot_linear.bias,
            self.humanNodeRNN.encoder_linear.weight, self.humanNodeRNN.encoder_linear.bias)
        m = masks.reshape(B)
        h_edge = rnn_hxs["human_human_edge_rnn"].reshape(B, self.num_edges, -1)
        h_node = rnn_hxs["human_node_rnn"].reshape(B, 1, -1)
        H = h_edge.shape[-1]
        if out_hxs is None:
            d_edge = torch.empty_like(h_edge)
            d_node = torch.empty_like(h_node)
        else:
            d_edge = out_hxs["human_human_edge_rnn"].view(B, self.num_edges, H)
            d_node = out_hxs["human_node_rnn"].view(B, 1, -1)
        if te.is_cuda and H % 32 == 0:
            # both edge RNNs in one launch, the input projections in the kernel (ops.gru_infer_group)
            gs, gt = self.humanhumanEdgeRNN_spatial.gru, self.humanhumanEdgeRNN_temporal.gru
            out_s, out_t = ops.gru_infer_group(
                (se.reshape(B * N, 64), h_edge[:, 1:, :], m, gs.weight_ih_l0, gs.weight_hh_l0, gs.bias_ih_l0,
                 gs.bias_hh_l0, d_edge[:, 1:, :]),
                (te.reshape(B, 64), h_edge[:, 0:1, :], m, gt.weight_ih_l0, gt.weight_hh_l0, gt.bias_ih_l0,
                 gt.bias_hh_l0, d_edge[:, 0:1, :]))
        else:
            out_t = self.humanhumanEdgeRNN_temporal.infer_step(te.reshape(B, 64), h_edge[:, 0:1, :], m,
                                                               d_edge[:, 0:1, :])
            out_s = self.humanhumanEdgeRNN_spatial.infer_step(se.reshape(B * N, 64), h_edge[:, 1:, :], m,
                                                              d_edge[:, 1:, :])
        weighted, _ = self.attn(out_t.view(1, B, H), out_s.view(1, B, N, H))
        outputs, _ = self.humanNodeRNN(ne.reshape(1, B, 64), out_t.view(1, B, H), weighted, h_node, m, dest=d_node)
        rnn_hxs["human_node_rnn"] = d_node
        rnn_hxs["human_human_edge_rnn"] = d_edge
        hidden_critic = self.critic(outputs)
        hidden_actor = self.actor(outputs)
        return self.critic_linear(hidden_critic).squeeze(0), hidden_actor.squeeze(0), rnn_hxs
