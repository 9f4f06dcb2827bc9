import builtins

import numpy as np


class Box(object):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is None:
            shape = np.shape(low)
        self.low = np.broadcast_to(np.asarray(low, dtype=np.float64), shape).astype(dtype)
        self.high = np.broadcast_to(np.asarray(high, dtype=np.float64), shape).astype(dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)


class Dict(object):
    def __init__(self, spaces):
        self.spaces = builtins.dict(spaces)   # a `gym.spaces.dict` submodule import shadows `dict` here
