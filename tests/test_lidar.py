"""LiDAR observation + ConvGRU policy vs the reference.

tests/golden/lidar_*.npz: states right after CrowdSimDict.reset() with robot.policy = 'convgru' and
lidar.enable, and the reference's (1, 187) observation (oracle/gen_golden.py gen_lidar; the reference's
`np.int` — removed in NumPy 1.24 — aliased to int while recording). tests/golden/convgru.npz: the
reference ConvGRU Policy on procedural weights.
Tolerances: the robot part and the scan are float64 -> float32 like the reference: exact on CPU (same
libm); on the GPU the trigonometry may differ in the last ulp, which can move a beam's first sample
inside the disc by one 0.01 m step (0.002 in the observation) or flip a beam at an obstacle's angular
edge; at most 0.5 % of beams may differ, by at most that much — everything else is bit-exact."""
import glob
import os

import numpy as np
import pytest
import torch

from tests import helpers as H
from tests.helpers import masked_gru_ref

LIDAR = sorted(os.path.basename(p) for p in glob.glob(os.path.join(H.GOLDEN, "lidar_*.npz")))


def _obs_cases(d):
    """(cfg, state of reset k-1 or None, state of reset k, reference obs of reset k): reset()'s observation
    carries the scan taken at the previous reset (zeros at the first)."""
    cfg = H.cn_config_from_meta(d)
    prev = None
    for k in range(int(d["resets"])):
        sv = H.state_from(d, "k%d_post_" % k, cfg)
        yield cfg, prev, sv, d["k%d_obs" % k]
        prev = sv


def _lidar_kw(d):
    return dict(beams=int(d["meta_num_beams"]), max_range=float(d["meta_max_range"]),
                robot_radius=float(d["meta_lidar_robot_radius"]))


@pytest.mark.parametrize("name", LIDAR)
def test_oracle_lidar_vs_reference(name):
    from oracle import lidar_ref

    d = H.load(name)
    kw = _lidar_kw(d)
    for cfg, prev, sv, want in _obs_cases(d):
        held = (np.zeros((sv.E, kw["beams"]), np.float32) if prev is None else
                lidar_ref.convgru_scans(prev, half_world=cfg.square_width / 2, **kw))
        got = lidar_ref.convgru_obs(sv, held, kw["max_range"])
        np.testing.assert_array_equal(got, want)


def _check_gpu_obs(got, want):
    np.testing.assert_array_equal(got[:, 0, :7], want[:, 0, :7])
    diff = np.abs(got[:, 0, 7:] - want[:, 0, 7:])
    # beams at full range read |1 - d/5| with d = |(c*5 + x) - x|: the last-ulp trig differences leave
    # values of ~1e-16 instead of 0 — numerically nothing; a beam counts as different above 1e-6
    bad = diff > 1e-6
    assert bad.mean() <= 0.005, "%.4f of beams differ (max %.3g): %s" % (bad.mean(), diff.max(),
                                                                          np.argwhere(bad)[:10].tolist())


@pytest.mark.gpu
@pytest.mark.parametrize("name", LIDAR)
def test_gpu_lidar_obs_vs_reference(name):
    from crowdnav_dsrnn_amd.engine import CrowdNavEngine

    d = H.load(name)
    kw = _lidar_kw(d)
    cfg = H.cn_config_from_meta(d)
    eng = CrowdNavEngine(cfg, "cuda:0")
    out = torch.zeros((cfg.num_envs, 1, 7 + kw["beams"]), device="cuda:0")
    lid = torch.zeros((cfg.num_envs, kw["beams"]), device="cuda:0")
    for _, prev, sv, want in _obs_cases(d):
        eng.set_state(sv)          # reset k: the observation carries the scan of reset k-1, then rescans
        eng.lidar_obs(out, lid, None, True, **kw)
        torch.cuda.synchronize()
        _check_gpu_obs(out.cpu().numpy(), want)
    eng.close()


@pytest.mark.gpu
def test_gpu_convgru_vecenv_scan_is_per_episode():
    """The VecEnv's 'convgru' observation: the scan only changes on the step AFTER an auto-reset (the reset
    observation carries the finished episode's scan; crowd_sim_dict.py:238-251 never refreshes it)."""
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv

    c = clone_config(Config())
    c.robot.policy = "convgru"
    c.lidar.enable = True
    c.sim.circle_radius = 7.0
    c.sim.human_num = 5
    c.action_space.kinematics = "holonomic"
    E = 64
    envs = CrowdNavVecEnv(c, E, 0, "cuda:0")
    assert tuple(envs.observation_space.shape) == (1, 187)
    o0 = envs.reset().clone()
    assert o0.shape == (E, 1, 187)
    g = torch.Generator(device="cuda:0").manual_seed(3)
    assert bool((o0[:, 0, 7:] == 0).all())      # first reset: no scan held yet
    scan = None
    prev_done = torch.ones(E, dtype=torch.bool, device="cuda:0")
    changed = 0
    for _ in range(60):
        a = torch.randn(E, 2, device="cuda:0", generator=g)
        o, r, done, *_ = envs.step_device(a)
        cur = o[:, 0, 7:].clone()
        if scan is not None:
            assert bool((cur == scan)[~prev_done].all())
            changed += int((cur != scan).any(1)[prev_done].sum())
        scan = cur
        prev_done = done.bool()
    assert changed > 0
    envs.close()


def _convgru_policy(device):
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.policy import Policy
    from crowdnav_dsrnn_amd.spaces import action_space, lidar_observation_space

    c = clone_config(Config())
    c.robot.policy = "convgru"
    pol = Policy(lidar_observation_space(180), action_space(), base="convgru", base_kwargs=c)
    pol.load_state_dict(H.procedural_state_dict(pol))
    return pol.to(device)


def _run_convgru(z, device):
    pol = _convgru_policy(device)
    t = lambda k: torch.from_numpy(z[k]).to(device)  # noqa: E731
    with torch.no_grad():
        v, a, lp, h = pol.act(t("act_obs"), t("act_hxs"), t("act_masks"), deterministic=True)
    v2, lp2, ent, h2 = pol.evaluate_actions(t("ev_obs"), t("act_hxs"), t("ev_masks"), t("ev_actions"))
    return [x.detach().cpu().numpy() for x in (v, a, lp, h, v2, lp2, ent, h2)]


_NAMES = ("act_value", "act_action", "act_logp", "act_hxs_out", "ev_value", "ev_logp", "ev_entropy", "ev_hxs_out")


def test_convgru_state_dict_keys():
    z = H.load("convgru.npz")
    assert sorted(_convgru_policy("cpu").state_dict().keys()) == [str(k) for k in z["state_dict_keys"]]


def test_convgru_policy_cpu_vs_reference(monkeypatch):
    from crowdnav_dsrnn_amd import ops

    monkeypatch.setattr(ops, "masked_gru", masked_gru_ref)
    z = H.load("convgru.npz")
    for n, got in zip(_NAMES, _run_convgru(z, "cpu")):
        np.testing.assert_allclose(got, z[n], atol=1e-5, rtol=1e-5, err_msg=n)


@pytest.mark.gpu
def test_convgru_policy_gpu_vs_reference():
    z = H.load("convgru.npz")
    for n, got in zip(_NAMES, _run_convgru(z, "cuda:0")):
        np.testing.assert_allclose(got, z[n], atol=1e-4, rtol=1e-4, err_msg=n)


@pytest.mark.gpu
def test_gpu_convgru_rollout_and_ppo_update():
    """train.py's ConvGRU branch on device: LiDAR VecEnv -> ConvGRU act -> RolloutStorage -> PPO update."""
    from crowdnav_dsrnn_amd.config import Config, clone_config
    from crowdnav_dsrnn_amd.envs import CrowdNavVecEnv
    from crowdnav_dsrnn_amd.learner import PPO
    from crowdnav_dsrnn_amd.learner.loop import RolloutTrainer
    from crowdnav_dsrnn_amd.learner.storage import RolloutStorage
    from crowdnav_dsrnn_amd.policy import Policy

    c = clone_config(Config())
    c.robot.policy = "convgru"
    c.lidar.enable = True
    c.sim.circle_radius = 7.0
    c.action_space.kinematics = "holonomic"
    c.ppo.num_steps = 8
    c.ppo.num_mini_batch = 2
    c.ppo.epoch = 2
    torch.manual_seed(0)
    envs = CrowdNavVecEnv(c, 32, 0, "cuda:0")
    pol = Policy(envs.observation_space, envs.action_space, base="convgru", base_kwargs=c).to("cuda:0")
    before = [p.detach().clone() for p in pol.parameters()]
    agent = PPO(pol, 0.2, c.ppo.epoch, c.ppo.num_mini_batch, 0.5, 0.0, lr=4e-5, eps=1e-5, max_grad_norm=0.5)
    tr = RolloutTrainer(c, envs, pol, agent)
    assert isinstance(tr.rollouts, RolloutStorage)
    st = tr.update()
    assert all(np.isfinite([st["value_loss"], st["action_loss"], st["dist_entropy"]]))
    assert any(not torch.equal(a, b) for a, b in zip(before, pol.parameters()))
    envs.close()
