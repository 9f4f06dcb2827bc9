"""Torch-facing wrappers of the native kernels (no compute in Python; the HIP kernels are mandatory).

edge_features(...)  — the fused DSRNN input layers (cn_edge_features, include/crowdnav.h): one launch
                      computes relu(temporal encoder), relu(spatial encoder) and
                      relu(node encoder(robot_linear(robot_node))) for every env (and time step).
"""
import torch

from . import _lib


class EdgeFeaturesUnavailable(RuntimeError):
    pass


def _stream(device):
    import ctypes

    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _c(t):
    return t.contiguous().float() if (not t.is_contiguous() or t.dtype != torch.float32) else t


class _EdgeFeatures(torch.autograd.Function):
    """Forward = fused HIP kernel. Backward = the matching gradients of the three tiny input layers
    (recomputed from the saved inputs with torch ops on the same device; these layers are
    <2% of the DSRNN FLOPs)."""

    @staticmethod
    def forward(ctx, robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn):
        E = temporal.shape[0]
        N = spatial.shape[1]
        dev = temporal.device
        t_out = torch.empty((E, 64), dtype=torch.float32, device=dev)
        s_out = torch.empty((E, N, 64), dtype=torch.float32, device=dev)
        n_out = torch.empty((E, 64), dtype=torch.float32, device=dev)
        args = [_c(x) for x in (robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn)]
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().cn_edge_features(_stream(dev), E, N, *[a.data_ptr() for a in args],
                                                   t_out.data_ptr(), s_out.data_ptr(), n_out.data_ptr()))
        ctx.save_for_backward(*args, t_out, s_out, n_out)
        return t_out, s_out, n_out

    @staticmethod
    def backward(ctx, g_t, g_s, g_n):
        robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn, t_out, s_out, n_out = ctx.saved_tensors
        E, N = temporal.shape[0], spatial.shape[1]
        x_t = temporal.reshape(E, 2)
        x_s = spatial.reshape(E * N, 2)
        x_r = robot_node.reshape(E, 7)
        gt = g_t * (t_out > 0)
        gs = (g_s * (s_out > 0)).reshape(E * N, 64)
        gn = g_n * (n_out > 0)
        h = x_r @ Wr.t() + br
        g_h = gn @ Wn
        grads = [
            (g_h @ Wr).reshape(robot_node.shape),
            (gt @ Wt).reshape(temporal.shape),
            (gs @ Ws).reshape(spatial.shape),
            gt.t() @ x_t, gt.sum(0), gs.t() @ x_s, gs.sum(0), g_h.t() @ x_r, g_h.sum(0), gn.t() @ h, gn.sum(0),
        ]
        return tuple(grads)


def edge_features(robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn):
    """robot_node (E,1,7) temporal (E,1,2) spatial (E,N,2) -> (E,64), (E,N,64), (E,64)."""
    if not robot_node.is_cuda:
        raise EdgeFeaturesUnavailable("the DSRNN edge-feature layers run only as the fused HIP kernel "
                                      "(tensors are on %s)" % robot_node.device)
    return _EdgeFeatures.apply(robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn)
