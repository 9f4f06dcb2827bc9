"""Agent policy plugin surface: `policy_factory[name](config).predict(JointState) -> ActionXY`.

Mirrors crowd_nav/policy/policy_factory.py:1-17: the reference's humans call
`policy.predict(JointState(self FullState, [ObservableState]))` once per human per step
(crowd_sim.py:1121-1161 -> human.py:11-20). Here 'orca' and 'social_force' run on the GPU through the
C ABI (`cn_orca_predict`: the step kernel's quad-cooperative RVO2 code path; `cn_social_force_predict`:
the step kernel's f64 social force), one launch per call; `predict_batch` takes many agents' states in
one launch (the MI355X-shaped use). 'none' returns None like the reference; 'srnn' / 'convgru' keep
SRNN.clip_action (crowd_nav/policy/srnn.py:18-48). Any other name is absent, as in the reference.

ORCA keeps the reference's per-object simulator semantics (orca.py:85-115): the simulator -- and with it
every agent's ORCA radius (radius + 0.01 + safety_space) and max speed (own v_pref, others 1) -- is
created at the first predict and only re-created when the number of agents changes; later calls only
update positions and velocities. RVO2 works in float32 (positions, velocities, radii, the preferred
velocity are cast at the boundary) and returns float32 velocities. Simulators of <= 10 agents run on the
engine's quad path (`cn_orca_predict`); 11 to 64 agents on the kd-tree path (`cn_orca_predict_kd`, RVO2's
KdTree neighbour order with the persisted agents_ permutation); more than 64 raise UnsupportedConfig.
"""
import collections
import ctypes

import numpy as np

from . import _lib
from .config import UnsupportedConfig

ActionXY = collections.namedtuple("ActionXY", ["vx", "vy"])      # crowd_sim/envs/utils/action.py:3
ActionRot = collections.namedtuple("ActionRot", ["v", "r"])      # crowd_sim/envs/utils/action.py:4


class FullState:
    """crowd_sim/envs/utils/state.py FullState(px, py, vx, vy, radius, gx, gy, v_pref, theta)."""

    def __init__(self, px, py, vx, vy, radius, gx, gy, v_pref, theta):
        self.px, self.py, self.vx, self.vy, self.radius = px, py, vx, vy, radius
        self.gx, self.gy, self.v_pref, self.theta = gx, gy, v_pref, theta
        self.position = (px, py)
        self.goal_position = (gx, gy)
        self.velocity = (vx, vy)


class ObservableState:
    """crowd_sim/envs/utils/state.py ObservableState(px, py, vx, vy, radius)."""

    def __init__(self, px, py, vx, vy, radius):
        self.px, self.py, self.vx, self.vy, self.radius = px, py, vx, vy, radius
        self.position = (px, py)
        self.velocity = (vx, vy)


class JointState:
    """crowd_sim/envs/utils/state.py JointState(self_state, human_states)."""

    def __init__(self, self_state, human_states):
        assert isinstance(self_state, FullState)
        for h in human_states:
            assert isinstance(h, ObservableState)
        self.self_state = self_state
        self.human_states = human_states


def _torch_stream():
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("agent policies run on the GPU (torch.cuda.is_available() is False)")
    dev = torch.device("cuda", torch.cuda.current_device())
    return torch, dev, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


MAX_ORCA_AGENTS = 64   # cn_orca_predict_kd's simulator size limit (include/crowdnav.h)


class Policy:
    """crowd_nav/policy/policy.py:5-19 (attributes the env sets: time_step, phase, env, ...)."""

    def __init__(self, config):
        self.trainable = False
        self.phase = None
        self.model = None
        self.device = None
        self.last_state = None
        self.time_step = None
        self.env = None
        self.config = config

    def predict(self, state):
        raise NotImplementedError

    @staticmethod
    def reach_destination(state):
        s = state.self_state
        return np.linalg.norm((s.py - s.gy, s.px - s.gx)) < s.radius


class ORCA(Policy):
    """crowd_nav/policy/orca.py:6-139 on the GPU (cn_orca_predict)."""

    def __init__(self, config):
        super().__init__(config)
        self.name = "ORCA"
        self.max_neighbors = None
        self.radius = None
        self.max_speed = 1
        # the simulator's state that outlives a predict (orca.py:85-115): agent count, frozen radii f32 [A],
        # self max speed f32, and RVO2's KdTree agent order (KdTree::agents_, re-permuted by every doStep's
        # tree build; it decides the order of equally distant neighbours when A > 10)
        self.sim = None

    def _frame(self, state):
        """float32 agents [A][5] (px, py, vx, vy, frozen radius) and [maxSpeed, pref.x, pref.y] of agent 0."""
        s, hs = state.self_state, state.human_states
        A = len(hs) + 1
        if A > MAX_ORCA_AGENTS:
            raise UnsupportedConfig("ORCA.predict: %d agents per simulator (the GPU predict serves <= %d)"
                                    % (A, MAX_ORCA_AGENTS))
        self.max_neighbors = len(hs)
        self.radius = s.radius
        if self.sim is not None and self.sim[0] != A:   # orca.py:85-90
            self.sim = None
        if self.sim is None:                            # orca.py:91-109: parameters frozen at creation
            safety = self.config.orca.safety_space
            radii = np.array([s.radius + 0.01 + safety] + [h.radius + 0.01 + safety for h in hs], np.float32)
            self.sim = (A, radii, np.float32(s.v_pref), np.arange(A, dtype=np.uint8))
        ag = np.zeros((A, 5), np.float32)
        ag[0, :4] = (s.px, s.py, s.vx, s.vy)
        for k, h in enumerate(hs):
            ag[k + 1, :4] = (h.px, h.py, h.vx, h.vy)
        ag[:, 4] = self.sim[1]
        v = np.array((s.gx - s.px, s.gy - s.py))     # orca.py:118-122
        speed = np.linalg.norm(v)
        pref = v / speed if speed > 1 else v
        return ag, np.array([self.sim[2], pref[0], pref[1]], np.float32)

    def predict(self, state):
        return predict_batch([self], [state])[0]


class SOCIAL_FORCE(Policy):
    """crowd_nav/policy/social_force.py:6-66 on the GPU (cn_social_force_predict, float64)."""

    def __init__(self, config):
        super().__init__(config)
        self.name = "social_force"

    def predict(self, state):
        return predict_batch([self], [state])[0]


class SRNN(Policy):
    """crowd_nav/policy/srnn.py:6-48: the robot policy placeholder of the env (the network is
    crowdnav_dsrnn_amd.policy.Policy); clip_action mutates raw_action in place like the reference."""

    def __init__(self, config):
        super().__init__(config)
        self.time_step = config.env.time_step
        self.name = "srnn" if config.robot.policy == "srnn" else config.robot.policy
        self.trainable = True
        self.multiagent_training = True

    def clip_action(self, raw_action, v_pref):
        if self.config.action_space.kinematics == "holonomic":
            n = np.linalg.norm(raw_action)
            if n > v_pref:
                raw_action[0] = raw_action[0] / n * v_pref
                raw_action[1] = raw_action[1] / n * v_pref
            return ActionXY(raw_action[0], raw_action[1])
        raw_action[0] = np.clip(raw_action[0], -0.1, 0.1)
        raw_action[1] = np.clip(raw_action[1], -0.1, 0.1)
        return ActionRot(raw_action[0], raw_action[1])

    def predict(self, state):
        raise NotImplementedError("the srnn robot is driven by the learner's actions (CrowdSimDict.step)")


def none_policy():
    return None


def predict_batch(policies, states):
    """predict() of many agents in one launch per policy kind: policies[i].predict(states[i]) for all i
    (ORCA agents grouped by simulator size). Returns a list of ActionXY (python floats)."""
    if len(policies) != len(states):
        raise ValueError("one state per policy")
    out = [None] * len(policies)
    torch, dev, st = None, None, None
    L = _lib.lib()
    orca_by_a, sf_by_m = {}, {}
    for i, (p, s) in enumerate(zip(policies, states)):
        if isinstance(p, ORCA):
            orca_by_a.setdefault(len(s.human_states) + 1, []).append(i)
        elif isinstance(p, SOCIAL_FORCE):
            sf_by_m.setdefault(len(s.human_states), []).append(i)
        else:
            raise TypeError("predict_batch: ORCA / SOCIAL_FORCE policies only, got %r" % type(p).__name__)
    if orca_by_a or sf_by_m:
        torch, dev, st = _torch_stream()
    for A, idx in orca_by_a.items():
        frames = [policies[i]._frame(states[i]) for i in idx]
        ag = torch.from_numpy(np.stack([f[0] for f in frames])).to(dev)
        sf = torch.from_numpy(np.stack([f[1] for f in frames])).to(dev)
        res = torch.zeros((len(idx), 4), dtype=torch.float32, device=dev)
        c = policies[idx[0]].config
        ts = policies[idx[0]].time_step or c.env.time_step
        if A > 10:   # KdTree path: each simulator's persisted agent order goes in and comes back re-permuted
            perm = torch.from_numpy(np.stack([policies[i].sim[3] for i in idx])).to(dev)
            _lib.check(L.cn_orca_predict_kd(st, len(idx), A, ag.data_ptr(), sf.data_ptr(),
                                            float(c.orca.neighbor_dist), float(c.orca.time_horizon), float(ts),
                                            perm.data_ptr(), res.data_ptr()))
            pn = perm.cpu().numpy()
            for k, i in enumerate(idx):
                policies[i].sim[3][:] = pn[k]
        else:
            _lib.check(L.cn_orca_predict(st, len(idx), A, ag.data_ptr(), sf.data_ptr(), float(c.orca.neighbor_dist),
                                         float(c.orca.time_horizon), float(ts), res.data_ptr()))
        r = res.cpu().numpy()
        for k, i in enumerate(idx):
            out[i] = ActionXY(float(r[k, 0]), float(r[k, 1]))
            policies[i].last_state = states[i]
    for M, idx in sf_by_m.items():
        selfs = np.array([[states[i].self_state.px, states[i].self_state.py, states[i].self_state.vx,
                           states[i].self_state.vy, states[i].self_state.radius, states[i].self_state.gx,
                           states[i].self_state.gy, states[i].self_state.v_pref, states[i].self_state.theta]
                          for i in idx], np.float64)
        oth = np.array([[[h.px, h.py, h.vx, h.vy, h.radius] for h in states[i].human_states] for i in idx],
                       np.float64).reshape(len(idx), M, 5)
        s_d = torch.from_numpy(selfs).to(dev)
        o_d = torch.from_numpy(np.ascontiguousarray(oth)).to(dev)
        res = torch.zeros((len(idx), 2), dtype=torch.float64, device=dev)
        c = policies[idx[0]].config
        _lib.check(L.cn_social_force_predict(st, len(idx), M, s_d.data_ptr(), o_d.data_ptr() if M else None,
                                             float(c.sf.A), float(c.sf.B), float(c.sf.KI), float(c.env.time_step),
                                             res.data_ptr()))
        r = res.cpu().numpy()
        for k, i in enumerate(idx):
            out[i] = ActionXY(float(r[k, 0]), float(r[k, 1]))
    return out


policy_factory = {"orca": ORCA, "none": none_policy, "social_force": SOCIAL_FORCE, "srnn": SRNN, "convgru": SRNN}
