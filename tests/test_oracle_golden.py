"""The CPU oracle (oracle/cpu_ref.c) against golden vectors recorded from the REFERENCE itself
(oracle/gen_golden.py runs the reference's CrowdSimDict through import shims). Pins the oracle
before it is trusted as the GPU checker."""
import glob
import os

import numpy as np
import pytest

from crowdnav_dsrnn_amd import abi
from tests import helpers as H

SPAWN = sorted(os.path.basename(p) for p in glob.glob(os.path.join(H.GOLDEN, "spawn_*.npz")))
ROLL = sorted(os.path.basename(p) for p in glob.glob(os.path.join(H.GOLDEN, "roll_*.npz")))


def test_fixtures_present():
    assert len(SPAWN) >= 8 and len(ROLL) >= 10, (SPAWN, ROLL)


def test_mt19937_matches_numpy(oracle):
    """numpy legacy RandomState is the reference's RNG (crowd_sim_dict.py:154)."""
    for seed in (0, 1, 2000, 2001, 123456789, 2**32 - 1):
        got = oracle.mt_draw(seed, 1500)
        want = np.random.RandomState(seed).random_sample(1500)
        assert np.array_equal(got, want), seed


@pytest.mark.parametrize("name", SPAWN)
def test_spawn_bit_exact(oracle, name):
    """CrowdSimDict.reset() states and first observations, bit-exact (tolerance 0)."""
    d = H.load(name)
    cfg = H.cn_config_from_meta(d)
    eng = oracle.RefEngine(cfg)
    for k in range(int(d["resets"])):
        pre = H.state_from(d, "k%d_pre_" % k, cfg)
        eng.set_state(pre)
        obs = eng.reset()
        errs = H.compare_state(eng.get_state(), d, "k%d_post_" % k, tol=0.0)
        assert not errs, errs
        for key, ok in (("robot_node", "robot_node"), ("temporal", "temporal_edges"), ("spatial", "spatial_edges")):
            assert np.array_equal(obs[ok].reshape(d["k%d_%s" % (k, key)].shape), d["k%d_%s" % (k, key)]), key


@pytest.mark.parametrize("name", ROLL)
def test_rollout_teacher_forced(oracle, name):
    """Teacher-forced CrowdSimDict.step + VecEnv auto-reset + Monitor: exact events/done/flags/indices,
    1e-5 on positions, rewards and observations (north-star tolerance)."""
    d = H.load(name)
    cfg = H.cn_config_from_meta(d)
    eng = oracle.RefEngine(cfg)
    errs = H.run_teacher_forced(eng, d, cfg, tol=H.POS_TOL)
    assert not errs, "\n".join(errs[:20])


def test_rollouts_cover_every_event():
    seen = set()
    for name in ROLL:
        seen |= set(np.unique(H.load(name)["event"]).tolist())
    assert seen == {abi.EV_NOTHING, abi.EV_DANGER, abi.EV_COLLISION, abi.EV_REACHGOAL, abi.EV_TIMEOUT}, seen
