"""Observation / action spaces of CrowdSimDict (crowd_sim/envs/crowd_sim_dict.py:31-69).

gym.spaces is used when gym is importable; otherwise these minimal stand-ins carry the same public
fields the callers read (`.spaces`, `.shape`, `.dtype`, `.low`, `.high`; the Policy checks the class
name 'Box', pytorchBaselines/a2c_ppo_acktr/model.py:36)."""
from collections import OrderedDict

import numpy as np

try:  # pragma: no cover - gym is absent in this image
    from gym.spaces import Box as _GymBox
    from gym.spaces import Dict as _GymDict
except Exception:  # noqa: BLE001
    _GymBox = _GymDict = None


class Box:
    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, dtype=self.dtype)
        self.high = np.full(self.shape, high, dtype=self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))

    def __repr__(self):
        return "Box(%s, %s)" % (self.shape, self.dtype)


class Dict:
    def __init__(self, spaces):
        self.spaces = OrderedDict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]

    def keys(self):
        return self.spaces.keys()

    def __repr__(self):
        return "Dict(" + ", ".join("%s:%r" % kv for kv in self.spaces.items()) + ")"


def _box(shape):
    if _GymBox is not None:  # pragma: no cover
        return _GymBox(low=-np.inf, high=np.inf, shape=shape, dtype=np.float32)
    return Box(-np.inf, np.inf, shape, np.float32)


def observation_space(human_num):
    """robot_node (1,7), temporal_edges (1,2), spatial_edges (N,2), float32, unbounded (crowd_sim_dict.py:31-56)."""
    d = OrderedDict([("robot_node", _box((1, 7))), ("temporal_edges", _box((1, 2))),
                     ("spatial_edges", _box((human_num, 2)))])
    return _GymDict(d) if _GymDict is not None else Dict(d)


def lidar_observation_space(num_beams):
    """The ConvGRU policy's observation: Box (1, 7 + num_beams) float32 (crowd_sim_dict.py:57-62)."""
    return _box((1, 7 + int(num_beams)))


def action_space():
    """Box(2,) float32, unbounded (crowd_sim_dict.py:64-69)."""
    return _box((2,))
