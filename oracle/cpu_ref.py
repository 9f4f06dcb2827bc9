"""ctypes wrapper of oracle/build/libcn_oracle.so (the C restatement in oracle/cpu_ref.c).

TEST INFRASTRUCTURE ONLY — see oracle/__init__.py. Mirrors the product engine's interface
(`reset` / `step` / `get_state` / `set_state`) on host numpy arrays.
"""
import ctypes
import os
import subprocess

import numpy as np

from crowdnav_dsrnn_amd import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libcn_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        build()   # make: a no-op when the library is newer than cpu_ref.c (never a stale checker)
        L = ctypes.CDLL(_LIB_PATH)
        vp, fp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float)
        L.cnref_create.argtypes = [ctypes.POINTER(abi.CnConfig), ctypes.POINTER(vp)]
        L.cnref_destroy.argtypes = [vp]
        L.cnref_state_bytes.argtypes = [vp]
        L.cnref_state_bytes.restype = ctypes.c_int64
        L.cnref_reset.argtypes = [vp, vp, vp, vp]
        L.cnref_step.argtypes = [vp] + [vp] * 10
        L.cnref_get_state.argtypes = [vp, vp]
        L.cnref_set_state.argtypes = [vp, vp]
        L.cnref_mt_draw.argtypes = [ctypes.c_uint32, ctypes.c_int, vp]
        L.cnref_philox_draw.argtypes = [ctypes.c_uint32, ctypes.c_int, vp]
        L.cnref_philox4x32_10.argtypes = [vp, vp, vp]
        L.cnref_rvo2_agent0.argtypes = [ctypes.c_int, vp, vp, vp, vp, vp, ctypes.c_float, ctypes.c_float,
                                        ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp, vp]
        L.cnref_set_threads.argtypes = [ctypes.c_int]
        L.cnref_set_rows.argtypes = [vp, vp]
        L.cnref_norm_zone_margin.restype = ctypes.c_double
        L.cnref_norm_zone_margin.argtypes = [ctypes.c_double] * 5 + [ctypes.c_int, ctypes.c_int]
        L.cnref_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class RefEngine:
    """E envs of the C restatement; host numpy in/out."""

    def __init__(self, cfg: abi.CnConfig):
        self.cfg = cfg.copy()
        self.E, self.N = cfg.num_envs, cfg.human_num
        h = ctypes.c_void_p()
        rc = lib().cnref_create(ctypes.byref(self.cfg), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(lib().cnref_last_error().decode())
        self.h = h
        self.nbytes = lib().cnref_state_bytes(h)

    def __del__(self):
        if getattr(self, "h", None) is not None and _lib is not None:
            _lib.cnref_destroy(self.h)
            self.h = None

    def _obs_bufs(self):
        return (np.zeros((self.E, 1, 7), np.float32), np.zeros((self.E, 1, 2), np.float32),
                np.zeros((self.E, self.N, 2), np.float32))

    def reset(self):
        rn, te, se = self._obs_bufs()
        lib().cnref_reset(self.h, _p(rn), _p(te), _p(se))
        return {"robot_node": rn, "temporal_edges": te, "spatial_edges": se}

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.E, 2)
        rn, te, se = self._obs_bufs()
        rew = np.zeros(self.E, np.float32)
        done = np.zeros(self.E, np.uint8)
        ev = np.zeros(self.E, np.int8)
        info = np.zeros((self.E, abi.INFO_K), np.float32)
        epr = np.zeros(self.E, np.float64)
        epl = np.zeros(self.E, np.int32)
        lib().cnref_step(self.h, _p(a), _p(rn), _p(te), _p(se), _p(rew), _p(done), _p(ev), _p(info), _p(epr), _p(epl))
        obs = {"robot_node": rn, "temporal_edges": te, "spatial_edges": se}
        return obs, rew, done.astype(bool), ev, info, epr, epl

    def get_state(self):
        buf = np.zeros(self.nbytes, np.uint8)
        lib().cnref_get_state(self.h, _p(buf))
        return abi.StateView(buf, self.E, self.N, self.cfg.robot_visible)

    def set_state(self, sv):
        assert sv.blob.nbytes == self.nbytes
        lib().cnref_set_state(self.h, _p(np.ascontiguousarray(sv.blob)))


class RefMixedEngine:
    """Oracle of the mixed engine (cn_create_mixed): one RefEngine per group whose env e is
    row rows[e] of the whole engine (seeds / round-robin scenarios from the global index), stepped on its
    rows' actions, outputs scattered back to the rows; spatial_edges padded to the largest human count
    with a never-seen human (the reference's unseen belief (15, 15), crowd_sim.py:437-455, relative to
    the robot's float64 position)."""

    def __init__(self, cfgs, env_group):
        eg = np.asarray(env_group, np.int32)
        self.E, self.N = int(eg.size), max(int(c.human_num) for c in cfgs)
        self.groups = []
        for g, c in enumerate(cfgs):
            rows = np.nonzero(eg == g)[0].astype(np.int32)
            if rows.size == 0:
                continue
            assert c.num_envs == rows.size
            eng = RefEngine(c)
            rc = lib().cnref_set_rows(eng.h, _p(rows))
            if rc != 0:
                raise RuntimeError(lib().cnref_last_error().decode())
            self.groups.append((eng, rows))

    def _scatter(self, parts, reset):
        E, N = self.E, self.N
        obs = {"robot_node": np.zeros((E, 1, 7), np.float32), "temporal_edges": np.zeros((E, 1, 2), np.float32),
               "spatial_edges": np.zeros((E, N, 2), np.float32)}
        outs = None
        for (eng, rows), p in zip(self.groups, parts):
            o = p if reset else p[0]
            obs["robot_node"][rows] = o["robot_node"]
            obs["temporal_edges"][rows] = o["temporal_edges"]
            obs["spatial_edges"][rows, :eng.N] = o["spatial_edges"]
            if eng.N < N:
                sv = eng.get_state()
                rx, ry = sv.r_px, sv.r_py
                obs["spatial_edges"][rows, eng.N:, 0] = (15.0 - rx).astype(np.float32)[:, None]
                obs["spatial_edges"][rows, eng.N:, 1] = (15.0 - ry).astype(np.float32)[:, None]
            if not reset:
                if outs is None:
                    outs = [np.zeros((E,) + a.shape[1:], a.dtype) for a in p[1:]]
                for dst, a in zip(outs, p[1:]):
                    dst[rows] = a
        return obs if reset else (obs,) + tuple(outs)

    def reset(self):
        return self._scatter([eng.reset() for eng, _ in self.groups], True)

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.float32).reshape(self.E, 2)
        return self._scatter([eng.step(a[rows]) for eng, rows in self.groups], False)

    def get_state(self):
        return [(rows, eng.get_state()) for eng, rows in self.groups]

    def set_state(self, svs):
        for (eng, rows), (rows2, sv) in zip(self.groups, svs):
            assert np.array_equal(rows, rows2)
            eng.set_state(sv)


def mt_draw(seed, n):
    out = np.zeros(n, np.float64)
    lib().cnref_mt_draw(seed, n, _p(out))
    return out


def philox_draw(key, n):
    """First n doubles of the CN_RNG_PHILOX stream of episode seed `key`."""
    out = np.zeros(n, np.float64)
    lib().cnref_philox_draw(key, n, _p(out))
    return out


def philox4x32_10(ctr, key):
    c, k = np.ascontiguousarray(ctr, np.uint32), np.ascontiguousarray(key, np.uint32)
    out = np.zeros(4, np.uint32)
    lib().cnref_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def norm_zone_margin(px, py, vx, vy, r, f32, lhs):
    """Signed distance of the robot's norm-zone predicate from its decision boundary (cpu_ref.c)."""
    return lib().cnref_norm_zone_margin(float(px), float(py), float(vx), float(vy), float(r), int(bool(f32)),
                                        int(lhs))


def rvo2_agent0(X, Y, VX, VY, R, vmax, pref, neighbor_dist=10.0, time_horizon=5.0, time_step=0.25, perm=None):
    A = len(X)
    f = lambda v: np.ascontiguousarray(v, np.float32)
    X, Y, VX, VY, R = map(f, (X, Y, VX, VY, R))
    out = np.zeros(2, np.float32)
    pp = None if perm is None else np.ascontiguousarray(perm, np.uint8)
    lib().cnref_rvo2_agent0(A, _p(X), _p(Y), _p(VX), _p(VY), _p(R), vmax, float(pref[0]), float(pref[1]),
                            neighbor_dist, time_horizon, time_step, _p(pp), _p(out))
    return out
