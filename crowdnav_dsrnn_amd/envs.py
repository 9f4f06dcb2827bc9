"""VecEnv drop-in for the reference's environment stack, backed by the batched HIP engine.

Reference stack this replaces:
    gym.make('CrowdSimDict-v0')                      crowd_sim/__init__.py:9-11
    make_env / make_vec_envs                         pytorchBaselines/a2c_ppo_acktr/envs.py:33-156
    bench.Monitor (episode r/l/t)                    baselines (external), consumed at train.py:266-267
    ShmemVecEnv / DummyVecEnv (auto-reset)           pytorchBaselines/a2c_ppo_acktr/shmem_vec_env.py:89-168
    VecPyTorch (torch obs, (E,1) reward)             pytorchBaselines/a2c_ppo_acktr/envs.py:208-239

`make_vec_envs(...)` keeps the reference signature and returns a `CrowdNavVecEnv` whose reset/step have
VecPyTorch's return types:
    reset()      -> {'robot_node' (E,1,7), 'temporal_edges' (E,1,2), 'spatial_edges' (E,N,2)} float32 on `device`
    step(action) -> obs dict on `device`, reward (E,1) float32 CPU tensor, done np.ndarray bool (E,),
                    infos: a tuple-like of E dicts {'info': step_info[, 'episode': {r, l, t}]}, built lazily
                    on access from the engine's event codes and metrics (events are info.py instances)
All env work runs on the GPU in one cn_step launch pair; there is no per-env Python and no CPU fallback.
`step_device(actions)` is the zero-copy variant for on-device rollouts (no host sync).

Sharding: `shard=(rank, world)` makes this process own the contiguous env block
[rank*E/world, (rank+1)*E/world) of the `num_processes` global envs, with the reference's global seed
schedule (thisSeed = seed + global index, nenv = num_processes), so a sharded run steps exactly the envs
an unsharded run would.
"""
import time

import numpy as np

from . import abi, info as info_mod, spaces
from .config import make_cn_config

_REGISTRY = {}


def register(id, entry_point):  # noqa: A002 - gym's keyword name
    """gym.envs.registration.register equivalent (crowd_sim/__init__.py:9-11): `entry_point` is a
    "module:Class" string (or the class) of a batched env with CrowdNavVecEnv's constructor; make_vec_envs
    resolves it like gym.make does. When gym itself is importable the id is registered there too, so
    `gym.spec(id)` / `gym.envs.registry` list it as the reference's registration does."""
    _REGISTRY[id] = entry_point
    try:
        import gym  # noqa: F401  (absent in this image; optional)
        from gym.envs.registration import register as gym_register
    except Exception:
        return
    try:
        gym_register(id=id, entry_point=entry_point)
    except Exception:   # already registered
        pass


def registry():
    return dict(_REGISTRY)


def resolve(env_name):
    """The registered entry point of `env_name` as a class (gym's load("module:attr"))."""
    if env_name not in _REGISTRY:
        raise KeyError("No registered env with id: %s (registered: %s)" % (env_name, sorted(_REGISTRY)))
    ep = _REGISTRY[env_name]
    if not isinstance(ep, str):
        return ep
    import importlib

    mod, _, attr = ep.partition(":")
    obj = importlib.import_module(mod)
    for a in attr.split("."):
        obj = getattr(obj, a)
    return obj


register("CrowdSimDict-v0", "crowdnav_dsrnn_amd.envs:CrowdNavVecEnv")


def make_vec_envs(env_name, seed, num_processes, gamma, log_dir, device, allow_early_resets,
                  num_frame_stack=None, config=None, ax=None, test_case=-1, fig=None, shard=None,
                  engine_device=None):
    """envs.py:106-156. `gamma` / `log_dir` are accepted for signature compatibility (VecNormalize only
    wraps Box observations, the Monitor writes no file: envs.py:79,141-146). `ax` / `fig` select the
    matplotlib rendering path, which is out of scope and rejected."""
    env_cls = resolve(env_name)
    if config is None:
        raise ValueError("config is required (CrowdSim.configure(config), envs.py:65)")
    if ax is not None or fig is not None:
        raise NotImplementedError("rendering (render_axis / render_figure / test_case) is out of scope")
    if num_frame_stack is not None:
        raise NotImplementedError("frame stacking applies to image observations only")
    rank, world = shard if shard is not None else (0, 1)
    if num_processes % world != 0:
        raise ValueError("num_processes=%d does not split over %d shards" % (num_processes, world))
    E = num_processes // world
    return env_cls(config, E, seed, device, allow_early_resets=allow_early_resets,
                   env_offset=rank * E, nenv=num_processes, engine_device=engine_device)


class _LazyInfos:
    """Tuple-like of E info dicts, each built on first access (train.py iterates them; most callers only
    read a few). Holds host copies of the step's event codes / metrics / Monitor counters."""

    def __init__(self, venv, event, done, info, ep_return, ep_len, t):
        self._v, self._event, self._done, self._info = venv, event, done, info
        self._ep_return, self._ep_len, self._t = ep_return, ep_len, t
        self._cache = [None] * len(event)

    def __len__(self):
        return len(self._cache)

    def _build(self, i):
        v, row = self._v, self._info[i]
        sc = v.scenario_names[int(row[abi.INFO_SCENARIO])]
        si = {"aggregate_nav_time": int(row[abi.INFO_AGG_NAV_TIME]),
              "path_violation": int(row[abi.INFO_PATH_VIOLATION])}
        if v.side_preference:
            si[sc] = {"left": int(row[abi.INFO_SIDE_LEFT]), "right": int(row[abi.INFO_SIDE_RIGHT])}
            si["separation"] = float(row[abi.INFO_SEPARATION])
        si["personal_violation"] = int(row[abi.INFO_PERSONAL_VIOLATION])
        si["jerk_cost"] = float(row[abi.INFO_JERK_COST])
        si["dist_to_goal"] = float(row[abi.INFO_DIST_TO_GOAL])
        si["speed_violation"] = int(row[abi.INFO_SPEED_VIOLATION])
        si["scenario"] = sc
        si["event"] = info_mod.make_event(int(self._event[i]), row[abi.INFO_MIN_DIST])
        d = {"info": si}
        if self._done[i]:
            d["episode"] = {"r": round(float(self._ep_return[i]), 6), "l": int(self._ep_len[i]), "t": self._t}
        return d

    def __getitem__(self, i):
        if isinstance(i, slice):
            return tuple(self[j] for j in range(*i.indices(len(self))))
        if i < 0:
            i += len(self)
        if self._cache[i] is None:
            self._cache[i] = self._build(i)
        return self._cache[i]

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


class _RobotView:
    """Read-only view of env i's robot (Agent attributes read by evaluation.py:206,284)."""

    def __init__(self, env):
        self._env = env

    def _s(self, name):
        return float(getattr(self._env._venv._state(), name)[self._env._i])

    time_step = property(lambda self: self._env.time_step)
    v_pref = property(lambda self: self._s("r_vpref"))
    radius = property(lambda self: self._s("r_radius"))
    px = property(lambda self: self._s("r_px"))
    py = property(lambda self: self._s("r_py"))
    gx = property(lambda self: self._s("r_gx"))
    gy = property(lambda self: self._s("r_gy"))
    vx = property(lambda self: self._s("r_vx"))
    vy = property(lambda self: self._s("r_vy"))
    theta = property(lambda self: self._s("r_theta"))

    @property
    def kinematics(self):
        return self._env._venv.config.action_space.kinematics


class _EnvView:
    """Stands in for `venv.envs[i].env` (the CrowdSimDict behind the Monitor; evaluation.py:71-251)."""

    def __init__(self, venv, i):
        self._venv, self._i = venv, i
        self.robot = _RobotView(self)

    @property
    def env(self):  # Monitor.env -> the CrowdSimDict
        return self

    global_time = property(lambda self: float(self._venv._state().gtime[self._i]))
    time_step = property(lambda self: float(self._venv.config.env.time_step))
    time_limit = property(lambda self: float(self._venv.config.env.time_limit))
    human_num = property(lambda self: int(self._venv.config.sim.human_num))
    thisSeed = property(lambda self: int(self._venv.cn_cfg.seed + self._venv.cn_cfg.env_offset + self._i))
    nenv = property(lambda self: int(self._venv.cn_cfg.nenv))
    phase = property(lambda self: self._venv.phase)

    @property
    def current_scenario(self):
        return self._venv.scenario_names[int(self._venv._state().scenario[self._i])]

    def render(self, *a, **k):
        raise NotImplementedError("rendering is out of scope")

    render_traj = render


class _VecView:
    def __init__(self, venv):
        self.envs = [_EnvView(venv, i) for i in range(venv.num_envs)]
        self.num_envs = venv.num_envs


class CrowdNavVecEnv:
    """E CrowdSimDict envs on one GPU with VecPyTorch/ShmemVecEnv/Monitor semantics."""

    def __init__(self, config, num_envs, seed, device, allow_early_resets=False, env_offset=0, nenv=None,
                 engine_device=None, phase=None):
        import torch

        from .engine import CrowdNavEngine

        self.torch = torch
        self.config = config
        self.num_envs = int(num_envs)
        nenv = self.num_envs if nenv is None else int(nenv)
        self.phase = phase if phase is not None else ("train" if nenv > 1 else "test")
        self.cn_cfg = make_cn_config(config, num_envs=self.num_envs, env_offset=env_offset, nenv=nenv,
                                     phase=self.phase,
                                     seed=seed if seed is not None else config.env.seed)
        self.device = torch.device(device)
        if engine_device is None and self.device.type == "cuda":
            engine_device = self.device
        self.engine = CrowdNavEngine(self.cn_cfg, engine_device)
        # 'convgru' observation (crowd_sim_dict.py:57-62, 96-101): robot state + the episode's LiDAR scan
        self.obs_mode = "convgru" if getattr(config.robot, "policy", "srnn") == "convgru" else "srnn"
        if self.obs_mode == "convgru":
            lc = dict(config.lidar.cfg)
            self._lidar_cfg = dict(enable=bool(config.lidar.enable), beams=int(lc["num_beams"]),
                                   max_range=float(lc["max_range"]), robot_radius=float(lc["robot_radius"]))
            B = self._lidar_cfg["beams"]
            self.observation_space = spaces.lidar_observation_space(B)
            self._lidar = torch.zeros((self.num_envs, B), dtype=torch.float32, device=self.engine.device)
            self._lidar_obs = torch.zeros((self.num_envs, 1, 7 + B), dtype=torch.float32, device=self.engine.device)
        else:
            self.observation_space = spaces.observation_space(int(config.sim.human_num))
        self.action_space = spaces.action_space()
        self.scenario_names = list(abi.SCENARIOS)
        self.side_preference = bool(config.test.side_preference)
        self.allow_early_resets = allow_early_resets
        self.venv = _VecView(self)
        self._tstart = time.time()
        self._was_reset = False
        self._state_cache = None
        self._pending = None
        E = self.num_envs
        pin = dict(pin_memory=True)
        self._h_reward = torch.empty((E,), dtype=torch.float32, **pin)
        self._h_done = torch.empty((E,), dtype=torch.uint8, **pin)
        self._h_event = torch.empty((E,), dtype=torch.int8, **pin)
        self._h_info = torch.empty((E, abi.INFO_K), dtype=torch.float32, **pin)
        self._h_epr = torch.empty((E,), dtype=torch.float64, **pin)
        self._h_epl = torch.empty((E,), dtype=torch.int32, **pin)

    # ---- VecEnv API --------------------------------------------------------------------------
    def _obs_out(self, o):
        if isinstance(o, dict):
            return {k: v.to(self.device, copy=True) for k, v in o.items()}
        return o.to(self.device, copy=True)

    def _convgru_obs(self, reset_mask):
        return self.engine.lidar_obs(self._lidar_obs, self._lidar, reset_mask, **self._lidar_cfg)

    def reset(self):
        """VecPyTorch.reset (envs.py:215-222). Monitor forbids a second reset of a running episode
        unless allow_early_resets (baselines bench.Monitor.reset)."""
        if self._was_reset and not self.allow_early_resets:
            raise RuntimeError("Tried to reset an environment before done. If you want to allow early resets, "
                               "wrap your env with Monitor(env, path, allow_early_resets=True)")
        self._was_reset = True
        self._state_cache = None
        o = self.engine.reset()
        if self.obs_mode == "convgru":
            o = self._convgru_obs(None)
        return self._obs_out(o)

    def step_async(self, actions):
        self._pending = actions

    def step_wait(self):
        if self._pending is None:
            raise RuntimeError("step_wait() without step_async()")
        actions, self._pending = self._pending, None
        obs, rew, done, ev, info, epr, epl = self.step_device(actions)
        t = self.torch
        for h, d in ((self._h_reward, rew), (self._h_done, done), (self._h_event, ev), (self._h_info, info),
                     (self._h_epr, epr), (self._h_epl, epl)):
            h.copy_(d, non_blocking=True)
        out_obs = self._obs_out(obs)
        t.cuda.current_stream(self.engine.device).synchronize()
        reward = self._h_reward.clone().unsqueeze(1)
        done_np = self._h_done.numpy().astype(bool)
        infos = _LazyInfos(self, self._h_event.numpy().copy(), done_np, self._h_info.numpy().copy(),
                           self._h_epr.numpy().copy(), self._h_epl.numpy().copy(),
                           round(time.time() - self._tstart, 6))
        return out_obs, reward, done_np, infos

    def step(self, actions):
        """VecPyTorch.step (envs.py:224-239) over CrowdSimDict.step + auto-reset + Monitor."""
        self.step_async(actions)
        return self.step_wait()

    def step_device(self, actions):
        """Zero-copy device step: actions (E,2) tensor/array -> the engine's output buffers
        (obs dict, reward (E,) f32, done (E,) u8, event (E,) i8, info (E,K) f32, ep_return f64, ep_len i32),
        all on the engine's GPU, valid until the next call. No host synchronisation."""
        t = self.torch
        if not isinstance(actions, t.Tensor):
            actions = t.as_tensor(np.asarray(actions, dtype=np.float32))
        self._state_cache = None
        out = self.engine.step(actions.reshape(self.num_envs, 2))
        if self.obs_mode == "convgru":
            out = (self._convgru_obs(out[2]),) + tuple(out[1:])
        return out

    def _state(self):
        if self._state_cache is None:
            self._state_cache = self.engine.get_state()
        return self._state_cache

    def render(self, *a, **k):
        raise NotImplementedError("rendering is out of scope")

    def render_traj(self, *a, **k):
        raise NotImplementedError("rendering is out of scope")

    def close(self):
        self.engine.close()

    @property
    def unwrapped(self):
        return self
