"""bench.py's measurement helpers (CPU): the algorithmic bytes per env-step of SURVEY §8d, the selection of
the counter profile (only a profile measured on a library built from exactly the current sources, on the
same workload, is ever reported -- a stale one never is), and the C5 mixed-engine configuration."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from crowdnav_dsrnn_amd import build  # noqa: E402


def test_algorithmic_bytes_survey_8d():
    assert bench.algorithmic_bytes_per_env_step(10) == 2274
    assert bench.algorithmic_bytes_per_env_step(25) == 5274
    assert bench.algorithmic_bytes_per_env_step(5) == 1274


def test_load_pmc_only_matches_current_sources(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    k = {"cn_step_kernel": {"hbm_bytes_per_launch": 1.0e7, "valu_issue_frac": 0.1, "avg_duration_ns": 5e4}}
    json.dump({"tag": "stale", "lib_src_hash": "0" * 64, "bench_args": "--steps 400", "kernels": k},
              open(prof / "pmc_stale.json", "w"))
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    assert bench.load_pmc("cn_step_kernel", "c2") is None
    json.dump({"tag": "good", "lib_src_hash": build.source_hash(), "bench_args": "--steps 400", "kernels": k},
              open(prof / "pmc_good.json", "w"))
    got = bench.load_pmc("cn_step_kernel", "c2")
    assert got["tag"] == "good" and got["traffic"] == 1.0e7
    assert bench.load_pmc("cn_step_kernel", "c3") is None   # measured on another workload


def test_c5_mixed_config_round_robin():
    cfgs, eg = bench.c5_mixed(8192, 0, 8192)
    assert [c.human_num for c in cfgs] == [5, 1]
    assert [c.num_envs for c in cfgs] == [int((eg == 0).sum()), int((eg == 1).sum())] == [3278, 4914]
    np.testing.assert_array_equal(eg, (np.arange(8192) % 5 >= 2).astype(np.int32))
    assert cfgs[1].side_preference == 1 and cfgs[1].circle_radius == 4 and cfgs[0].norm_zones == 1
