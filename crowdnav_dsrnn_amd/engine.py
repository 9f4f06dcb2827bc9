"""Device-resident batched CrowdSimDict engine (torch tensors in, torch tensors out).

Thin host wrapper over the C ABI (include/crowdnav.h, crowdnav_dsrnn_amd/csrc/cn_engine.hip): it
owns the output buffers (torch, on the engine's device) and passes `data_ptr()`s and the current
torch stream to `cn_reset` / `cn_step`. No compute happens here and there is no CPU fallback.
"""
import ctypes

import numpy as np

from . import _lib, abi


class CrowdNavEngine:
    """E environments of the reference's CrowdSimDict on one GPU.

    reset()                  -> obs dict (robot_node (E,1,7), temporal_edges (E,1,2), spatial_edges (E,N,2))
    step(actions (E,2) f32)  -> obs, reward (E,), done (E,) uint8, event (E,) int8, info (E,K), ep_return (E,) f64,
                                ep_len (E,) i32       (auto-reset of finished envs, like the reference VecEnv)
    Returned tensors are the engine's own buffers (overwritten by the next call); clone to keep them.
    """

    def __init__(self, cfg, device=None, _mixed=None):
        import torch

        self.torch = torch
        if not torch.cuda.is_available():
            raise RuntimeError("CrowdNavEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device if device is not None else "cuda:%d" % torch.cuda.current_device())
        L = _lib.lib()
        h = ctypes.c_void_p()
        if _mixed is None:
            self.cfg = cfg.copy()
            self.groups = None
            self.E, self.N = int(cfg.num_envs), int(cfg.human_num)
            _lib.check(L.cn_config_validate(ctypes.byref(self.cfg)))
            with torch.cuda.device(self.device):
                _lib.check(L.cn_create(ctypes.byref(self.cfg), self.device.index, ctypes.byref(h)))
        else:
            cfgs, env_group = _mixed
            arr = (abi.CnConfig * len(cfgs))(*[c.copy() for c in cfgs])
            for c in arr:
                if c.num_envs > 0:
                    _lib.check(L.cn_config_validate(ctypes.byref(c)))
            eg = np.ascontiguousarray(env_group, dtype=np.int32)
            self.E, self.N = int(eg.size), max(int(c.human_num) for c in cfgs)
            with torch.cuda.device(self.device):
                _lib.check(L.cn_create_mixed(arr, len(cfgs), eg.ctypes.data_as(ctypes.c_void_p), self.E,
                                             self.device.index, ctypes.byref(h)))
            self.cfg = arr[0].copy()
            self.groups = [(arr[g], np.nonzero(eg == g)[0].astype(np.int32)) for g in range(len(cfgs))
                           if (eg == g).any()]
        self._h = h
        nb = ctypes.c_int64()
        _lib.check(L.cn_state_bytes(h, ctypes.byref(nb)))
        self.state_bytes = nb.value
        E, N, dev = self.E, self.N, self.device
        hn = np.zeros(E, np.int32)
        _lib.check(L.cn_env_humans(h, hn.ctypes.data_as(ctypes.c_void_p)))
        self.env_humans = torch.from_numpy(hn).to(dev)            # (E,) humans of each env
        self.human_mask = torch.arange(N, device=dev)[None, :] < self.env_humans[:, None]   # (E, N) real slots
        self.robot_node = torch.zeros((E, 1, 7), dtype=torch.float32, device=dev)
        self.temporal_edges = torch.zeros((E, 1, 2), dtype=torch.float32, device=dev)
        self.spatial_edges = torch.zeros((E, N, 2), dtype=torch.float32, device=dev)
        self.reward = torch.zeros((E,), dtype=torch.float32, device=dev)
        self.done = torch.zeros((E,), dtype=torch.uint8, device=dev)
        self.event = torch.zeros((E,), dtype=torch.int8, device=dev)
        self.info = torch.zeros((E, abi.INFO_K), dtype=torch.float32, device=dev)
        self.ep_return = torch.zeros((E,), dtype=torch.float64, device=dev)
        self.ep_len = torch.zeros((E,), dtype=torch.int32, device=dev)
        self._step_args = None   # cached output pointers of step() (the buffers above are never reallocated)
        self._seq_fn = None

    @classmethod
    def mixed(cls, cfgs, env_group, device=None):
        """One engine over envs of several configurations (cn_create_mixed): env r runs
        cfgs[env_group[r]] (its own human count, scenarios, radius, ...). N = the largest human count;
        spatial_edges rows past an env's own count are padding (`human_mask` False): a never-seen human
        at the reference's unseen-belief position (15, 15). Build the configs with
        config.make_mixed_cn_configs."""
        return cls(None, device, _mixed=(list(cfgs), env_group))

    # -------------------------------------------------------------------------------------------
    def _stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def obs(self):
        return {"robot_node": self.robot_node, "temporal_edges": self.temporal_edges,
                "spatial_edges": self.spatial_edges}

    def reset(self):
        with self.torch.cuda.device(self.device):
            _lib.check(_lib.lib().cn_reset(self._h, self._stream(), self.robot_node.data_ptr(),
                                           self.temporal_edges.data_ptr(), self.spatial_edges.data_ptr()))
        return self.obs()

    def step(self, actions):
        t = self.torch
        if actions.device != self.device or actions.dtype != t.float32 or not actions.is_contiguous():
            actions = actions.to(device=self.device, dtype=t.float32).contiguous()
        if actions.numel() != self.E * 2:
            raise ValueError("actions must have E*2 = %d elements, got %d" % (self.E * 2, actions.numel()))
        # host cost per call matters when a short window starts on an idle GPU: the output pointers and the
        # bound C function are cached, and the device guard is entered only when another device is current
        if self._step_args is None:
            self.step_args()
        if t.cuda.current_device() == self.device.index:
            rc = self._step_fn(self._h, t.cuda.current_stream().cuda_stream, actions.data_ptr(), *self._step_args)
        else:
            with t.cuda.device(self.device):
                rc = self._step_fn(self._h, t.cuda.current_stream().cuda_stream, actions.data_ptr(), *self._step_args)
        _lib.check(rc)
        return self.obs(), self.reward, self.done, self.event, self.info, self.ep_return, self.ep_len

    def step_seq(self, actions):
        """T steps with actions (T, E, 2) f32 (a contiguous device tensor; views along T are fine) issued back to
        back from native code (cn_step_seq); returns the outputs of the last step, like step()."""
        t = self.torch
        if actions.device != self.device or actions.dtype != t.float32 or actions.dim() != 3:
            raise ValueError("step_seq: actions must be a float32 (T, E, 2) tensor on %s" % self.device)
        T = actions.shape[0]
        if tuple(actions.shape[1:]) != (self.E, 2) or actions.stride(2) != 1 or actions.stride(1) != 2:
            raise ValueError("step_seq: actions (T, E, 2) with each step's (E, 2) rows contiguous required")
        if self._step_args is None:
            self.step_args()
        if self._seq_fn is None:
            self._seq_fn = _lib.lib().cn_step_seq
        stride = actions.stride(0) if T > 1 else 2 * self.E
        if t.cuda.current_device() == self.device.index:
            rc = self._seq_fn(self._h, t.cuda.current_stream().cuda_stream, T, actions.data_ptr(), stride, *self._step_args)
        else:
            with t.cuda.device(self.device):
                rc = self._seq_fn(self._h, t.cuda.current_stream().cuda_stream, T, actions.data_ptr(), stride,
                                  *self._step_args)
        _lib.check(rc)
        return self.obs(), self.reward, self.done, self.event, self.info, self.ep_return, self.ep_len

    def step_args(self):
        """The output pointers of step() / step_seq() (cached: the buffers are never reallocated)."""
        if self._step_args is None:
            self._step_fn = _lib.lib().cn_step
            self._step_args = (self.robot_node.data_ptr(), self.temporal_edges.data_ptr(),
                               self.spatial_edges.data_ptr(), self.reward.data_ptr(), self.done.data_ptr(),
                               self.event.data_ptr(), self.info.data_ptr(), self.ep_return.data_ptr(),
                               self.ep_len.data_ptr())
        return self._step_args

    def set_graph_mode(self, on=True):
        """cn_set_graph_mode: keep the step sequence on the device so that step() can be captured in a
        torch.cuda.CUDAGraph (synchronises the current stream)."""
        with self.torch.cuda.device(self.device):
            _lib.check(_lib.lib().cn_set_graph_mode(self._h, self._stream(), int(bool(on))))

    # -------------------------------------------------------------------------------------------
    def lidar_obs(self, out, lidar, reset_mask=None, enable=True, beams=180, max_range=5.0, robot_radius=0.3):
        """The ConvGRU observation (cn_lidar_obs) into out (E,1,7+beams) f32; lidar (E,beams) f32 holds the
        per-episode scans and is refreshed where reset_mask (E,) u8 is set (None = every env)."""
        t = self.torch
        with t.cuda.device(self.device):
            _lib.check(_lib.lib().cn_lidar_obs(self._h, self._stream(),
                                               None if reset_mask is None else reset_mask.data_ptr(),
                                               int(bool(enable)), int(beams), float(max_range), float(robot_radius),
                                               lidar.data_ptr(), out.data_ptr()))
        return out

    def get_state(self):
        """abi.StateView of the engine; a mixed engine: [(rows, StateView of the group)] in group order."""
        buf = np.zeros(self.state_bytes, np.uint8)
        with self.torch.cuda.device(self.device):
            _lib.check(_lib.lib().cn_get_state(self._h, self._stream(), buf.ctypes.data_as(ctypes.c_void_p), 1))
        if self.groups is None:
            return abi.StateView(buf, self.E, self.N, self.cfg.robot_visible)
        out, off = [], 0
        for c, rows in self.groups:
            nb = abi.state_layout(int(c.num_envs), int(c.human_num), c.robot_visible)[1]
            out.append((rows, abi.StateView(buf[off:off + nb].copy(), int(c.num_envs), int(c.human_num),
                                            c.robot_visible)))
            off += nb
        return out

    def set_state(self, sv):
        if self.groups is not None:
            blob = np.concatenate([np.ascontiguousarray(v.blob).view(np.uint8).ravel() for _, v in sv])
        else:
            blob = np.ascontiguousarray(sv.blob)
        if blob.nbytes != self.state_bytes:
            raise ValueError("state blob has %d bytes, engine expects %d" % (blob.nbytes, self.state_bytes))
        with self.torch.cuda.device(self.device):
            _lib.check(_lib.lib().cn_set_state(self._h, self._stream(), blob.ctypes.data_as(ctypes.c_void_p), 1))

    def set_spawn_budget(self, cycles):
        """Test hook (cn_debug_set_spawn_budget): clock cycles a kd-tree-path spawning wave works per launch
        before it parks its spawn (default 600000; 0 = never). Results do not depend on it (round 5 fixed a rare
        case where they did: DESIGN.md)."""
        _lib.check(_lib.lib().cn_debug_set_spawn_budget(self._h, int(cycles)))

    def spawn_stats(self):
        """Cumulative spawn counters (cn_debug_spawn_stats; synchronises): kd-tree path spawns parked before
        starting, parked mid-way, resumed, completed by a resume; auto-resets drawn inline (no pending spawn)."""
        out = (ctypes.c_uint32 * 5)()
        _lib.check(_lib.lib().cn_debug_spawn_stats(self._h, out))
        return dict(zip(("parked_unstarted", "parked_midway", "resumed", "completed_on_resume", "inline_resets"),
                        list(out)))

    def close(self):
        if getattr(self, "_h", None) is not None:
            _lib.lib().cn_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class NumpyEngine:
    """numpy-in/numpy-out facade over CrowdNavEngine with the oracle's interface (used by tests)."""

    def __init__(self, cfg, device=None):
        self.eng = CrowdNavEngine(cfg, device)
        self.E, self.N = self.eng.E, self.eng.N

    def reset(self):
        o = self.eng.reset()
        self.eng.torch.cuda.synchronize(self.eng.device)
        return {k: v.cpu().numpy() for k, v in o.items()}

    def step(self, actions):
        t = self.eng.torch
        a = t.from_numpy(np.ascontiguousarray(actions, np.float32).reshape(self.E, 2)).to(self.eng.device)
        obs, rew, done, ev, info, epr, epl = self.eng.step(a)
        t.cuda.synchronize(self.eng.device)
        return ({k: v.cpu().numpy() for k, v in obs.items()}, rew.cpu().numpy(), done.cpu().numpy(),
                ev.cpu().numpy(), info.cpu().numpy(), epr.cpu().numpy(), epl.cpu().numpy())

    def get_state(self):
        return self.eng.get_state()

    def set_state(self, sv):
        self.eng.set_state(sv)
