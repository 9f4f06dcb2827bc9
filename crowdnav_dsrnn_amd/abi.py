"""ctypes mirror of include/crowdnav.h and include/crowdnav_state.h.

Pure data definitions (no compute): the `cn_config` struct, the enum values, and the state-blob
layout used by `cn_get_state` / `cn_set_state`. Shared by the product bindings
(`crowdnav_dsrnn_amd._lib`) and the test harness.
"""
import ctypes

import numpy as np

# --- enums (include/crowdnav.h) -------------------------------------------------------------------
HOLONOMIC, UNICYCLE = 0, 1
POLICY_ORCA, POLICY_SOCIAL_FORCE = 0, 1
PHASE_TRAIN, PHASE_VAL, PHASE_TEST = 0, 1, 2
PHASES = {"train": PHASE_TRAIN, "val": PHASE_VAL, "test": PHASE_TEST}
SCMODE_ROUND_ROBIN, SCMODE_SEQUENTIAL = 0, 1
RNG_MT19937, RNG_PHILOX = 0, 1   # include/crowdnav.h CN_RNG_*
RNG_MODE = {"mt19937": RNG_MT19937, "philox": RNG_PHILOX}

SCENARIOS = [
    "circle_crossing",
    "square_crossing",
    "parallel_traffic",
    "perpendicular_traffic",
    "side_pref_passing",
    "side_pref_overtaking",
    "side_pref_crossing",
]
SCENARIO_ID = {name: i for i, name in enumerate(SCENARIOS)}

EV_NOTHING, EV_DANGER, EV_COLLISION, EV_REACHGOAL, EV_TIMEOUT = 0, 1, 2, 3, 4

INFO_AGG_NAV_TIME = 0
INFO_PATH_VIOLATION = 1
INFO_PERSONAL_VIOLATION = 2
INFO_JERK_COST = 3
INFO_DIST_TO_GOAL = 4
INFO_SPEED_VIOLATION = 5
INFO_MIN_DIST = 6
INFO_SCENARIO = 7
INFO_SIDE_LEFT = 8
INFO_SIDE_RIGHT = 9
INFO_SEPARATION = 10
INFO_OVERFLOW = 11
INFO_K = 12

MAX_SCENARIOS = 8
MT_N = 624


class CnConfig(ctypes.Structure):
    """struct cn_config (include/crowdnav.h)."""

    _fields_ = [
        ("num_envs", ctypes.c_int32),
        ("human_num", ctypes.c_int32),
        ("env_offset", ctypes.c_int64),
        ("nenv", ctypes.c_int64),
        ("seed", ctypes.c_int64),
        ("phase", ctypes.c_int32),
        ("kinematics", ctypes.c_int32),
        ("human_policy", ctypes.c_int32),
        ("scenario_mode", ctypes.c_int32),
        ("num_scenarios", ctypes.c_int32),
        ("scenarios", ctypes.c_int32 * MAX_SCENARIOS),
        ("val_size", ctypes.c_int32),
        ("test_size", ctypes.c_int32),
        ("time_step", ctypes.c_double),
        ("time_limit", ctypes.c_double),
        ("circle_radius", ctypes.c_double),
        ("square_width", ctypes.c_double),
        ("robot_radius", ctypes.c_double),
        ("robot_vpref", ctypes.c_double),
        ("robot_fov", ctypes.c_double),
        ("human_radius", ctypes.c_double),
        ("human_vpref", ctypes.c_double),
        ("human_fov", ctypes.c_double),
        ("robot_visible", ctypes.c_int32),
        ("randomize_attributes", ctypes.c_int32),
        ("random_goal_changing", ctypes.c_int32),
        ("end_goal_changing", ctypes.c_int32),
        ("random_radii", ctypes.c_int32),
        ("random_v_pref", ctypes.c_int32),
        ("goal_change_chance", ctypes.c_double),
        ("end_goal_change_chance", ctypes.c_double),
        ("success_reward", ctypes.c_double),
        ("collision_penalty", ctypes.c_double),
        ("discomfort_dist", ctypes.c_double),
        ("discomfort_penalty_factor", ctypes.c_double),
        ("potential_factor", ctypes.c_double),
        ("norm_zone_penalty", ctypes.c_double),
        ("potential_based", ctypes.c_int32),
        ("time_factor", ctypes.c_int32),
        ("norm_zones", ctypes.c_int32),
        ("norm_zone_lhs", ctypes.c_int32),
        ("min_personal_space", ctypes.c_double),
        ("max_walking_speed", ctypes.c_double),
        ("social_metrics", ctypes.c_int32),
        ("side_preference", ctypes.c_int32),
        ("orca_neighbor_dist", ctypes.c_double),
        ("orca_safety_space", ctypes.c_double),
        ("orca_time_horizon", ctypes.c_double),
        ("orca_time_horizon_obst", ctypes.c_double),
        ("sf_A", ctypes.c_double),
        ("sf_B", ctypes.c_double),
        ("sf_KI", ctypes.c_double),
        ("max_tries", ctypes.c_int32),
        ("rng_mode", ctypes.c_int32),
    ]

    def copy(self):
        c = CnConfig()
        ctypes.memmove(ctypes.byref(c), ctypes.byref(self), ctypes.sizeof(CnConfig))
        return c


# --- state blob (include/crowdnav_state.h) ---------------------------------------------------------
CNT_ENV, CNT_HUM, CNT_PERM, CNT_MT = 0, 1, 2, 3
_T = {0: np.float64, 1: np.float32, 2: np.int64, 3: np.int32, 4: np.uint32, 5: np.uint8}

# (name, numpy dtype, count kind) in X-macro order — must match CN_STATE_FIELDS.
STATE_FIELDS = [
    ("r_px", 0, CNT_ENV), ("r_py", 0, CNT_ENV), ("r_gx", 0, CNT_ENV), ("r_gy", 0, CNT_ENV),
    ("r_vx", 0, CNT_ENV), ("r_vy", 0, CNT_ENV), ("r_theta", 0, CNT_ENV), ("r_dv", 0, CNT_ENV),
    ("r_radius", 0, CNT_ENV), ("r_vpref", 0, CNT_ENV), ("potential", 0, CNT_ENV), ("gtime", 0, CNT_ENV),
    ("last_ax", 0, CNT_ENV), ("last_ay", 0, CNT_ENV), ("ep_return", 0, CNT_ENV),
    ("case_counter", 2, CNT_ENV), ("ep_len", 3, CNT_ENV), ("scenario", 3, CNT_ENV),
    ("reset_count", 3, CNT_ENV), ("flags", 4, CNT_ENV), ("overflow", 4, CNT_ENV), ("mt_pos", 3, CNT_ENV),
    ("h_px", 0, CNT_HUM), ("h_py", 0, CNT_HUM), ("h_gx", 0, CNT_HUM), ("h_gy", 0, CNT_HUM),
    ("h_vx", 0, CNT_HUM), ("h_vy", 0, CNT_HUM), ("h_r", 0, CNT_HUM), ("h_vpref", 0, CNT_HUM),
    ("h_theta", 0, CNT_HUM),
    ("b_px", 0, CNT_HUM), ("b_py", 0, CNT_HUM), ("b_vx", 0, CNT_HUM), ("b_vy", 0, CNT_HUM), ("b_r", 0, CNT_HUM),
    ("o_r", 1, CNT_HUM), ("o_vmax", 1, CNT_HUM), ("o_dmask", 4, CNT_HUM),
    ("o_perm", 5, CNT_PERM),
    ("mt", 4, CNT_MT),
]
FLAG_ORCA_FROZEN = 0x1
FLAG_NAN = 0x2
FLAG_ROBOT_F32 = 0x4


def sim_agents(N, robot_visible):
    return N + (1 if robot_visible else 0)


def count_of(kind, N, robot_visible):
    A = sim_agents(N, robot_visible)
    if kind == CNT_ENV:
        return 1
    if kind == CNT_HUM:
        return N
    if kind == CNT_PERM:
        return N * A if A > 10 else 0
    return MT_N


def state_layout(E, N, robot_visible):
    """Return ({name: (offset, dtype, per_env_count)}, total_bytes) — mirrors cn_state_layout()."""
    off = 0
    out = {}
    for name, t, kind in STATE_FIELDS:
        off = (off + 255) & ~255
        dt = np.dtype(_T[t])
        cnt = count_of(kind, N, robot_visible)
        out[name] = (off, dt, cnt)
        off += E * cnt * dt.itemsize
    return out, (off + 255) & ~255


class StateView:
    """Named numpy views over a state blob (host bytes / numpy uint8 array)."""

    def __init__(self, blob, E, N, robot_visible):
        self.E, self.N, self.robot_visible = E, N, robot_visible
        self.layout, self.nbytes = state_layout(E, N, robot_visible)
        if blob is None:
            blob = np.zeros(self.nbytes, dtype=np.uint8)
        self.blob = blob
        assert self.blob.nbytes == self.nbytes, (self.blob.nbytes, self.nbytes)
        kinds = {name: kind for name, _, kind in STATE_FIELDS}
        for name, (off, dt, cnt) in self.layout.items():
            arr = self.blob[off:off + E * cnt * dt.itemsize].view(dt)
            if kinds[name] != CNT_ENV:
                arr = arr.reshape(E, cnt)
            setattr(self, name, arr)

    def copy(self):
        return StateView(self.blob.copy(), self.E, self.N, self.robot_visible)
