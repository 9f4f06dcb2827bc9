"""CN_RNG_PHILOX fast mode: the oracle's Philox4x32-10 against the published Random123
known-answer vectors, the stream conversion against an independent numpy Philox, and distribution-level
checks of resets / goal changes against the MT19937 parity mode (which is itself pinned bit-exact to
the reference by tests/test_oracle_golden.py)."""
import numpy as np
import pytest
from scipy import stats

from crowdnav_dsrnn_amd import abi
from crowdnav_dsrnn_amd.config import Config, clone_config, make_cn_config

# Random123 kat_vectors, philox4x32 R=10: counter (4 words), key (2 words) -> output (4 words)
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def np_philox(ctr0, k0, k1):
    """Vectorised Philox4x32-10 (counter (ctr0, 0, 0, 0)) in numpy uint64 arithmetic."""
    M = np.uint64(0xFFFFFFFF)
    x0 = np.asarray(ctr0, np.uint64)
    x1 = np.zeros_like(x0)
    x2 = np.zeros_like(x0)
    x3 = np.zeros_like(x0)
    k0, k1 = np.uint64(k0), np.uint64(k1)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * x0
        p1 = np.uint64(0xCD9E8D57) * x2
        x0, x1, x2, x3 = ((p1 >> np.uint64(32)) ^ x1 ^ k0) & M, p1 & M, ((p0 >> np.uint64(32)) ^ x3 ^ k1) & M, p0 & M
        k0, k1 = (k0 + np.uint64(0x9E3779B9)) & M, (k1 + np.uint64(0xBB67AE85)) & M
    return np.stack([x0, x1, x2, x3], -1).astype(np.uint32)


def test_philox_known_answers(oracle):
    for ctr, key, want in KAT:
        assert oracle.philox4x32_10(ctr, key).tolist() == list(want)
        if ctr[1:] == (0, 0, 0):
            assert np_philox([ctr[0]], key[0], key[1])[0].tolist() == list(want)


def test_philox_stream_conversion(oracle):
    """double k of episode seed s = words (2k, 2k+1) of philox(counter 2k >> 2) under key (s, 0x43726f77),
    converted like numpy's random_sample."""
    for seed in (0, 1, 2000, 123456789, 2 ** 32 - 1):
        n = 1001
        got = oracle.philox_draw(seed, n)
        q = 2 * np.arange(n)
        w = np_philox(q >> 2, seed, 0x43726F77).astype(np.int64)
        o = (q & 3)
        a = w[np.arange(n), o] >> 5
        b = w[np.arange(n), o + 1] >> 6
        want = (a * 67108864.0 + b) / 9007199254740992.0
        assert np.array_equal(got, want), seed
        assert got.min() >= 0 and got.max() < 1


def _cfg(E, rng, N=10, kin="unicycle", scen="circle_crossing", **over):
    c = clone_config(Config())
    c.sim.human_num = N
    c.action_space.kinematics = kin
    c.sim.train_val_sim = c.sim.test_sim = [scen]
    for k, v in over.items():
        sec, fld = k.split("__")
        setattr(getattr(c, sec), fld, v)
    return make_cn_config(c, num_envs=E, rng=rng)


def test_rng_mode_plumbing():
    assert _cfg(4, "mt19937").rng_mode == abi.RNG_MT19937
    assert _cfg(4, "philox").rng_mode == abi.RNG_PHILOX
    c = clone_config(Config())
    c.env.rng = "philox"
    assert make_cn_config(c, num_envs=2).rng_mode == abi.RNG_PHILOX
    from crowdnav_dsrnn_amd.config import UnsupportedConfig
    with pytest.raises(UnsupportedConfig):
        _cfg(4, "xorshift")


def _spawn_sample(oracle, rng, kin, scen, E=3000):
    eng = oracle.RefEngine(_cfg(E, rng, kin=kin, scen=scen))
    eng.reset()
    s = eng.get_state()
    out = {n: np.asarray(getattr(s, n), np.float64).reshape(-1)
           for n in ("r_px", "r_py", "r_gx", "r_gy", "r_theta", "h_px", "h_py", "h_gx", "h_gy", "h_r", "h_vpref")}
    return out, s


@pytest.mark.parametrize("kin,scen", [("unicycle", "circle_crossing"), ("holonomic", "square_crossing"),
                                      ("holonomic", "perpendicular_traffic")])
def test_philox_spawn_distributions_match_parity_mode(oracle, kin, scen):
    """Every spawn marginal (robot start/goal/heading, human start/goal/radius/v_pref) of 3,000 resets:
    two-sample Kolmogorov-Smirnov against the MT19937 mode (= the reference's draws)."""
    mt, _ = _spawn_sample(oracle, "mt19937", kin, scen)
    ph, s = _spawn_sample(oracle, "philox", kin, scen)
    for k in mt:
        if np.ptp(mt[k]) == 0:
            assert np.array_equal(mt[k], ph[k]), k
            continue
        p = stats.ks_2samp(mt[k], ph[k]).pvalue
        assert p > 1e-3, (k, p)
        assert not np.array_equal(mt[k], ph[k]), k   # a different stream, not the same draws
    # philox state: the key (episode seed) in mt[0], the word position, nothing else
    mtw = np.asarray(s.mt).reshape(s.E, -1)
    assert np.all(mtw[:, 1:] == 0)
    # one key per env (crowd_sim_dict.py:154: seed = counter_offset + case_counter + thisSeed)
    assert len(np.unique(mtw[:, 0])) == s.E
    assert np.all(np.asarray(s.mt_pos) > 0) and np.all(np.asarray(s.mt_pos) % 2 == 0)


def test_philox_episode_statistics_match_parity_mode(oracle):
    """A 160-step C2-shaped rollout of 1,024 envs (goal changes, auto-resets) under the same actions:
    outcome counts, goal-change-driven goal displacement and episode lengths agree in distribution."""
    res = {}
    for rng in ("mt19937", "philox"):
        eng = oracle.RefEngine(_cfg(1024, rng))
        eng.reset()
        r = np.random.RandomState(3)
        ev_counts = np.zeros(5, np.int64)
        lens, goal_moves = [], []
        prev = eng.get_state()
        for t in range(160):
            a = r.uniform(-0.1, 0.1, (1024, 2)).astype(np.float32)
            obs, rew, done, ev, info, epr, epl = eng.step(a)
            s = eng.get_state()
            ev_counts += np.bincount(ev.astype(np.int64), minlength=5)[:5]
            lens += list(np.asarray(epl)[done.astype(bool)])
            keep = ~done.astype(bool)
            d = np.hypot(np.asarray(s.h_gx) - np.asarray(prev.h_gx), np.asarray(s.h_gy) - np.asarray(prev.h_gy))
            goal_moves.append(d.reshape(1024, -1)[keep].reshape(-1))
            prev = s
        gm = np.concatenate(goal_moves)
        res[rng] = (ev_counts, np.asarray(lens), gm[gm > 0])
    (e0, l0, g0), (e1, l1, g1) = res["mt19937"], res["philox"]
    print("events", e0, e1, "episodes", len(l0), len(l1), "goal changes", len(g0), len(g1))
    # outcome frequencies (danger / collision / success / timeout) over ~160k env-steps
    chi = stats.chi2_contingency(np.stack([e0[1:], e1[1:]]) + 1)
    assert chi.pvalue > 1e-3, (e0, e1, chi.pvalue)
    assert stats.ks_2samp(l0, l1).pvalue > 1e-3, (l0.mean(), l1.mean())
    assert abs(len(g0) - len(g1)) < 5 * np.sqrt(len(g0)), (len(g0), len(g1))   # goal-change counts
    assert stats.ks_2samp(g0, g1).pvalue > 1e-3
