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


def test_launch_plan_never_reports_one_gpu_for_n():
    """`bench.py --gpus N` without a launcher starts N ranks itself; under a launcher --gpus must equal
    WORLD_SIZE (envs.py:120-139 builds the whole worker pool from one call)."""
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"})[0] == "error"
    assert bench.launch_plan(1, {"WORLD_SIZE": "2"})[0] == "error"
    assert bench.launch_plan(0, {})[0] == "error"


def test_single_command_two_rank_launch_gloo(tmp_path):
    """`python bench.py --gpus 2` (no WORLD_SIZE) spawns two ranks through torch.distributed.run; with the
    --dry-run hook each rank joins a gloo group and rank 0 prints n_gpus = 2 (no GPU touched)."""
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--dry-run"], env=env, capture_output=True, text=True,
                       timeout=240, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["max_over_ranks"] == 2.0
    # a mismatching launcher is refused (exit 2), not reported as a smaller run
    env2 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    q = subprocess.run([sys.executable, os.path.join(os.path.dirname(bench.__file__), "bench.py"), "--gpus", "2",
                        "--dry-run"], env=env2, capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert q.returncode == 2 and "WORLD_SIZE" in q.stderr


def test_window_object_arithmetic_and_fields():
    """env_window_obj (the main window, steady_state and the side_c3 / side_c5 objects): value = all ranks'
    env-steps / the window's max-over-ranks wall time, ms_per_step, the kernel time, resets, the wall-time
    breakdown and the HBM roofline of the step kernel from the algorithmic bytes."""
    m = {"workload": "c3", "W": 100, "K": 200, "launch": "cn_step_seq", "E_total": 4096, "N": 25,
         "bpl": bench.algorithmic_bytes_per_env_step(25) * 4096,
         "main": (0.11, 0.0005, 7219, 0.02)}
    o = bench.env_window_obj(m, world=2)
    assert o["value"] == round(2 * 4096 * 200 / 0.11, 1)
    assert o["ms_per_step"] == round(0.11 / 200 * 1e3, 6) and o["step_kernel_ms"] == 0.5
    assert o["launches"] == [100, 200] and o["resets"] == 7219 and o["window"] == "launches 101..300 after cn_reset"
    assert o["window_ms"]["wall"] == 110.0 and o["window_ms"]["step_kernels"] == 100.0
    r = o["roofline"]
    assert r["bound"] == "hbm" and r["algorithmic_bytes_per_launch"] == 5274 * 4096
    assert abs(r["achieved"] - 5274 * 4096 / 0.0005 / 1e9) < 1e-3 and r["peak"] == 8000.0


def test_side_windows_are_the_survey_shapes():
    """The default line's side windows: C3 and C5 after 100 warm-up launches over 200 timed ones, C4 one eager
    update + the graph-capturing one, then 2 timed updates, all inside the watchdog's deadline."""
    assert [w[0] for w in bench.SIDE_WINDOWS] == ["c3", "c5", "c4"]
    assert dict((w[0], w[1:]) for w in bench.SIDE_WINDOWS) == {"c3": (100, 200), "c5": (100, 200), "c4": (2, 2)}
    assert 0 < bench.SIDE_DEADLINE_S <= 300
