"""Shared test helpers: build engine configs from fixture metadata, move fixture states into blobs,
compare states with the tolerances the north star fixes (bit-exact on indices/flags/events;
1e-5 on positions and rewards)."""
import os
import zlib

import numpy as np

from crowdnav_dsrnn_amd import abi
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# f64 state fields compared with an absolute tolerance (positions, velocities, rewards ...)
FLOAT_FIELDS = {n for n, t, _ in abi.STATE_FIELDS if t in (0, 1)}
EXACT_FIELDS = {"case_counter", "ep_len", "scenario", "reset_count", "flags", "mt_pos", "o_dmask", "o_perm"}
POS_TOL = 1e-5


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


def ref_config(meta):
    c = clone_config(Config())
    c.action_space.kinematics = str(meta["meta_kinematics"])
    c.humans.policy = str(meta["meta_policy"])
    sc = str(meta["meta_scenarios"]).split(",")
    c.sim.train_val_sim = sc
    c.sim.test_sim = sc
    c.sim.human_num = int(meta["meta_N"])
    c.robot.FOV = float(meta["meta_robot_fov"])
    c.humans.FOV = float(meta["meta_human_fov"])
    c.test.side_preference = bool(meta["meta_side_pref"])
    c.test.social_metrics = bool(meta["meta_social_metrics"])
    c.robot.visible = bool(meta["meta_robot_visible"])
    c.humans.random_radii = bool(meta["meta_random_radii"])
    c.humans.random_v_pref = bool(meta["meta_random_v_pref"])
    c.reward.time_factor = bool(meta["meta_time_factor"])
    c.env.time_step = float(meta["meta_time_step"])
    c.reward.discomfort_penalty_factor = 10 * c.env.time_step
    c.sim.circle_radius = float(meta["meta_circle_radius"])
    if c.test.side_preference:
        c.humans.random_goal_changing = False
        c.humans.end_goal_changing = False
    c.reward.norm_zones = bool(meta["meta_norm_zones"])
    return c


def cn_config_from_meta(meta, E=None):
    c = ref_config(meta)
    E = int(meta["meta_E"]) if E is None else E
    return make_cn_config(c, num_envs=E, nenv=int(meta["meta_E"]))


def state_from(d, prefix, cfg, mt=None):
    sv = abi.StateView(None, cfg.num_envs, cfg.human_num, cfg.robot_visible)
    for name, _, _ in abi.STATE_FIELDS:
        key = prefix + name
        if key in d:
            getattr(sv, name)[...] = d[key].reshape(getattr(sv, name).shape)
    if mt is not None:
        sv.mt[...] = mt
    return sv


def mt_crc(sv):
    return np.array([zlib.crc32(np.ascontiguousarray(sv.mt[e]).tobytes()) for e in range(sv.E)], np.uint32)


def compare_state(got, d, prefix, tol=POS_TOL, skip=(), env_mask=None, where=""):
    """Compare a StateView with fixture fields `prefix+name`; returns list of mismatch strings."""
    errs = []
    for name, _, _ in abi.STATE_FIELDS:
        if name in skip or name == "mt" or (prefix + name) not in d:
            continue
        a = np.asarray(getattr(got, name))
        b = d[prefix + name].reshape(a.shape)
        if env_mask is not None:
            a, b = a[env_mask], b[env_mask]
        if name in EXACT_FIELDS:
            bad = a != b
        else:
            af, bf = a.astype(np.float64), b.astype(np.float64)
            bad = ~((np.abs(af - bf) <= tol) | (np.isnan(af) & np.isnan(bf)) | (af == bf))
        if bad.any():
            idx = np.argwhere(bad)[:3]
            errs.append("%s%s: %d mismatches, e.g. %s got=%s want=%s" % (
                where, name, int(bad.sum()), idx.tolist(), a[tuple(idx[0])], b[tuple(idx[0])]))
    if (prefix + "mt_crc") in d:
        c = mt_crc(got)
        want = d[prefix + "mt_crc"]
        if env_mask is not None:
            c, want = c[env_mask], want[env_mask]
        if (c != want).any():
            errs.append("%smt stream: %d envs differ" % (where, int((c != want).sum())))
    return errs


def at(d, prefix, t):
    """Slice step t out of stacked fixture fields `prefix*` -> {prefix+name: value}."""
    return {k: v[t] for k, v in d.items() if k.startswith(prefix)}


def compare_step(t, d, obs, rew, done, ev, info, epr, epl, tol=POS_TOL):
    errs = []
    for key, ok in (("robot_node", "robot_node"), ("temporal", "temporal_edges"), ("spatial", "spatial_edges")):
        a = np.asarray(obs[ok]).reshape(d[key][t].shape).astype(np.float64)
        b = d[key][t].astype(np.float64)
        if not np.allclose(a, b, atol=tol, rtol=0):
            i = np.unravel_index(np.argmax(np.abs(a - b)), a.shape)
            errs.append("t=%d obs %s max err %g at %s" % (t, key, np.abs(a - b).max(), i))
    if not np.array_equal(np.asarray(done).astype(np.uint8), d["done"][t]):
        errs.append("t=%d done %s vs %s" % (t, np.asarray(done).astype(int), d["done"][t]))
    if not np.array_equal(np.asarray(ev), d["event"][t]):
        errs.append("t=%d event %s vs %s" % (t, np.asarray(ev), d["event"][t]))
    if not np.allclose(np.asarray(rew, np.float64), d["reward"][t].astype(np.float64), atol=tol, rtol=0):
        errs.append("t=%d reward %s vs %s" % (t, rew, d["reward"][t]))
    dm = d["done"][t].astype(bool)
    if dm.any():
        if not np.allclose(np.asarray(epr)[dm], d["ep_return"][t][dm], atol=1e-4, rtol=0):
            errs.append("t=%d ep_return %s vs %s" % (t, np.asarray(epr)[dm], d["ep_return"][t][dm]))
        if not np.array_equal(np.asarray(epl)[dm], d["ep_len"][t][dm]):
            errs.append("t=%d ep_len %s vs %s" % (t, np.asarray(epl)[dm], d["ep_len"][t][dm]))
    want = d["info"][t]
    got = np.asarray(info)
    for k in (abi.INFO_AGG_NAV_TIME, abi.INFO_PERSONAL_VIOLATION, abi.INFO_SPEED_VIOLATION, abi.INFO_SCENARIO,
              abi.INFO_SIDE_LEFT, abi.INFO_SIDE_RIGHT):
        if not np.array_equal(got[:, k], want[:, k]):
            errs.append("t=%d info[%d] %s vs %s" % (t, k, got[:, k], want[:, k]))
    for k in (abi.INFO_DIST_TO_GOAL, abi.INFO_SEPARATION, abi.INFO_JERK_COST):
        if not np.allclose(got[:, k], want[:, k], atol=1e-4, rtol=1e-5):
            errs.append("t=%d info[%d] %s vs %s" % (t, k, got[:, k], want[:, k]))
    dg = np.asarray(ev) == abi.EV_DANGER
    if dg.any() and not np.allclose(got[dg, abi.INFO_MIN_DIST], want[dg, abi.INFO_MIN_DIST], atol=tol):
        errs.append("t=%d danger min_dist %s vs %s" % (t, got[dg, abi.INFO_MIN_DIST], want[dg, abi.INFO_MIN_DIST]))
    return errs


def run_teacher_forced(eng, d, cfg, tol=POS_TOL, max_errs=20, check_path_violation=True):
    """Teacher-forced replay of a roll_*.npz fixture on an engine exposing set_state/step/get_state.
    Before step t the engine gets the reference's post-state of step t-1 (its own MT19937 words are
    carried forward: the fixture stores a CRC of the reference stream, checked every step)."""
    errs = []
    T = d["actions"].shape[0]
    st = state_from(d, "init_", cfg)
    pv_mismatch = 0
    for t in range(T):
        eng.set_state(st)
        obs, rew, done, ev, info, epr, epl = eng.step(d["actions"][t])
        got = eng.get_state()
        errs += compare_step(t, d, obs, rew, done, ev, info, epr, epl, tol)
        errs += compare_state(got, at(d, "post_", t), "post_", tol, where="t=%d " % t)
        pv_mismatch += int((np.asarray(info)[:, abi.INFO_PATH_VIOLATION] != d["info"][t][:, abi.INFO_PATH_VIOLATION]).sum())
        if len(errs) >= max_errs:
            break
        st = state_from(at(d, "post_", t), "post_", cfg, mt=got.mt)
    if check_path_violation and pv_mismatch:
        errs.append("path_violation mismatches: %d" % pv_mismatch)
    return errs


# ---- DSRNN policy fixtures (tests/golden/dsrnn.npz, generated by oracle/gen_golden.py:gen_dsrnn) ----
def procedural_state_dict(model):
    """Same deterministic weights the fixture generator loaded into the reference Policy
    (oracle/gen_golden.py:procedural_state_dict): sorted key p ~ RandomState(1000+p).uniform(+-1/sqrt(fan_in))."""
    import math

    import torch

    out = {}
    for p, (k, v) in enumerate(sorted(model.state_dict().items())):
        shape = tuple(v.shape)
        s = 1.0 / math.sqrt(shape[-1] if len(shape) > 1 else 1)
        out[k] = torch.from_numpy(np.random.RandomState(1000 + p).uniform(-s, s, shape).astype(np.float32))
    return out


class BoxSpace:
    """Stand-in for gym.spaces.Box (only the class name and shape are read by Policy)."""

    def __init__(self, shape):
        self.shape = shape


BoxSpace.__name__ = "Box"


def make_policy(N, E=4, T=8, device="cpu"):
    from crowdnav_dsrnn_amd.policy import Policy

    c = clone_config(Config())
    c.sim.human_num = N
    c.training.num_processes = E
    c.ppo.num_steps = T
    c.ppo.num_mini_batch = 1
    pol = Policy({}, BoxSpace((2,)), base="srnn", base_kwargs=c)
    pol.load_state_dict(procedural_state_dict(pol))
    return pol.to(device).eval()


def edge_features_fp32(robot_node, temporal, spatial, Wt, bt, Ws, bs, Wr, br, Wn, bn):
    """Plain PyTorch fp32 restatement of the fused input layers (srnn_model.py:160-161, 210-211, 466)."""
    import torch

    E, N = temporal.shape[0], spatial.shape[1]
    t = torch.relu(temporal.reshape(E, 2) @ Wt.t() + bt)
    s = torch.relu(spatial.reshape(E * N, 2) @ Ws.t() + bs).reshape(E, N, 64)
    n = torch.relu((robot_node.reshape(E, 7) @ Wr.t() + br) @ Wn.t() + bn)
    return t, s, n


def masked_gru_ref(x, h0, masks, w_ih, w_hh, b_ih, b_hh):
    """Plain PyTorch fp32 restatement of the mask-segmented GRU (srnn_model.py:52-104): per step
    h <- h * mask[t], then torch.gru_cell (nn.GRU's cell)."""
    import torch

    outs = []
    h = h0
    for t in range(x.shape[0]):
        h = torch.gru_cell(x[t], h * masks[t].unsqueeze(-1), w_ih, w_hh, b_ih, b_hh)
        outs.append(h)
    return torch.stack(outs, 0), h


def gru_infer_step_ref(x, h0, m, w_ih, w_hh, b_ih, b_hh, dest):
    """Plain PyTorch restatement of ops.gru_infer_step: one masked GRU cell step over grouped rows,
    the new state also written into dest."""
    import torch

    h0g = h0 if h0.dim() == 3 else h0.unsqueeze(1)
    R, G, H = h0g.shape
    hm = (h0g * m.reshape(R, 1, 1)).reshape(R * G, H)
    h = torch.gru_cell(x.reshape(R * G, -1), hm, w_ih, w_hh, b_ih, b_hh)
    if dest is not None:
        (dest if dest.dim() == 3 else dest.unsqueeze(1)).copy_(h.view(R, G, H))
    return h


def attention_pool_ref(hs, attn):
    """Plain PyTorch restatement of EdgeAttention's weighted sum (srnn_model.py:320-333)."""
    import torch

    return torch.bmm(hs.transpose(1, 2), attn).squeeze(-1)
