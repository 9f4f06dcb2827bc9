"""C-ABI boundary checks that run without a GPU: the native library loads, exports every symbol
include/crowdnav.h declares, and agrees with the Python layout mirror (no compute calls)."""
import ctypes
import os
import re

import pytest

from crowdnav_dsrnn_amd import abi, _lib
from crowdnav_dsrnn_amd.config import Config, UnsupportedConfig, clone_config, make_cn_config

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(REPO, "include", "crowdnav.h")).read()
    return sorted(set(re.findall(r"\b(cn_[a-z_0-9]+)\s*\(", txt)) - {"cn_engine"})


@pytest.fixture(scope="module")
def L():
    from crowdnav_dsrnn_amd import build

    build.build()
    return _lib.lib()


def test_header_declares_expected_api():
    assert set(declared_symbols()) == set(_lib.EXPORTED)


def test_library_exports_every_declared_symbol(L):
    for sym in declared_symbols():
        assert hasattr(L, sym), sym


@pytest.mark.parametrize("cname,py", [("cn_gru_seq_fwd", _lib.GruSeqFwd), ("cn_gru_seq_bwd", _lib.GruSeqBwd),
                                      ("cn_gru_step_seg", _lib.GruStepSeg)])
def test_gru_seq_structs_match_header(cname, py):
    """The ctypes mirrors of the sequence-GRU argument structs list the header's fields in its order (every
    field 8 bytes: int64_t or a pointer, so the order fixes the layout)."""
    txt = open(os.path.join(REPO, "include", "crowdnav.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (cname, cname), txt, re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    fields = re.findall(r"(\w+)\s*;", body)
    assert fields == [f for f, _ in py._fields_]
    assert ctypes.sizeof(py) == 8 * len(fields)


def test_gru_seq_rejects_bad_arguments_without_launching(L):
    segs = (_lib.GruSeqFwd * 3)()
    assert L.cn_gru_fwd_seq(None, 4, 256, 3, segs) != 0      # at most two GRUs per call
    assert L.cn_gru_fwd_seq(None, 4, 96 + 4, 1, segs) != 0   # H % 32
    assert L.cn_gru_fwd_seq(None, 4, 256, 1, segs) != 0      # B = 0, null operands
    bsegs = (_lib.GruSeqBwd * 2)()
    bsegs[0].B, bsegs[1].B = 20480, 2048
    # workspace: bias partials of 128-row tiles ((160 + 16) x 4H per step) + the reduction's 64 x 4H
    assert L.cn_gru_bwd_seq_work_elems(3, 256, 2, bsegs) == (3 * 176 + 64) * 1024
    bsegs[0].B = 2048   # 16 x 4 tiles of 128 rows < 256 CUs: split-K on 32-row tiles (64 per step)
    assert L.cn_gru_bwd_seq_work_elems(2, 128, 1, bsegs) == (2 * 64 + 64) * 512
    assert L.cn_gru_bwd_seq(None, 0, 256, 1, bsegs, None, 0) != 0     # T = 0
    assert L.cn_gru_bwd_seq(None, 4, 256, 1, bsegs, None, 0) != 0
    assert b"cn_gru_bwd_seq" in L.cn_last_error()
    # a workspace below the size for the current device is rejected before any launch (the split-K
    # choice follows the device's CU count; dummy 16-byte aligned operands are never dereferenced)
    one = (_lib.GruSeqBwd * 1)()
    one[0] = _lib.GruSeqBwd(2048, 16, 32, 48, 64, 80, 96, 112, 128, 144)
    need = L.cn_gru_bwd_seq_work_elems(2, 128, 1, one)
    assert L.cn_gru_bwd_seq(None, 2, 128, 1, one, 4096, need - 1) != 0
    assert b"workspace smaller" in L.cn_last_error()
    # masked-state ring: nh >= 2 when T > 1 (a step reads hm[t % nh] while other workgroups write
    # hm[(t + 1) % nh]); nh == T with save (the backward reads every step's hm). Rejected before any launch
    # (non-null dummy addresses, 16-byte aligned, are never dereferenced)
    seg = (_lib.GruSeqFwd * 1)()
    seg[0] = _lib.GruSeqFwd(64, 16, 32, 48, 64, 80, 96, None, 1, None, None, None, 0)
    assert L.cn_gru_fwd_seq(None, 4, 256, 1, seg) != 0 and b"nh >= 2" in L.cn_last_error()
    seg[0].nh, seg[0].save = 2, 112
    assert L.cn_gru_fwd_seq(None, 4, 256, 1, seg) != 0 and b"nh == T" in L.cn_last_error()


def test_step_seq_and_graph_census_reject_bad_arguments(L):
    """cn_step_seq / cn_graph_node_counts validate their arguments before touching the GPU."""
    assert L.cn_step_seq(None, None, 4, None, 0, *([None] * 9)) != 0
    counts = (ctypes.c_int64 * 4)()
    assert L.cn_graph_node_counts(None, counts, 4, None) != 0
    assert L.cn_graph_node_counts(ctypes.c_void_p(16), counts, 33, None) != 0   # n > 32


def test_config_struct_size_matches(L):
    # a validate call on a deliberately invalid config only reads the struct (no GPU work)
    c = abi.CnConfig()
    assert L.cn_config_validate(ctypes.byref(c)) != 0
    assert b"num_envs" in L.cn_last_error()


def test_state_layout_matches_python_mirror(L):
    cfg = make_cn_config(clone_config(Config()), num_envs=37)
    for N, vis in ((5, 0), (10, 0), (12, 0), (25, 1), (1, 0)):
        cfg.human_num, cfg.robot_visible = N, vis
        offs = (ctypes.c_int64 * 64)()
        tot = ctypes.c_int64()
        assert L.cn_state_layout_offsets(ctypes.byref(cfg), offs, ctypes.byref(tot)) == 0
        lay, total = abi.state_layout(37, N, vis)
        assert total == tot.value
        for k, (name, _, _) in enumerate(abi.STATE_FIELDS):
            assert lay[name][0] == offs[k], name
            nm, tc, ck = ctypes.c_char_p(), ctypes.c_int(), ctypes.c_int()
            assert L.cn_state_field_info(k, ctypes.byref(nm), ctypes.byref(tc), ctypes.byref(ck)) == 0
            assert nm.value.decode() == name


def test_validate_rejects_unsupported(L):
    cfg = make_cn_config(clone_config(Config()), num_envs=8)
    assert L.cn_config_validate(ctypes.byref(cfg)) == 0
    bad = cfg.copy()
    bad.human_num = 40
    assert L.cn_config_validate(ctypes.byref(bad)) != 0
    bad = cfg.copy()
    bad.potential_based = 0
    assert L.cn_config_validate(ctypes.byref(bad)) != 0


def test_make_cn_config_rejects_unsupported_reference_options():
    c = clone_config(Config())
    c.sim.group_human = True
    with pytest.raises(UnsupportedConfig):
        make_cn_config(c, 4)
    c = clone_config(Config())
    c.robot.policy = "cadrl"
    with pytest.raises(UnsupportedConfig):
        make_cn_config(c, 4)
    c = clone_config(Config())        # the LiDAR / ConvGRU observation is served (cn_lidar_obs)
    c.lidar.enable = True
    c.robot.policy = "convgru"
    make_cn_config(c, 4)


def test_make_cn_config_defaults_follow_make_env():
    c = make_cn_config(clone_config(Config()), num_envs=12)
    assert c.phase == abi.PHASE_TRAIN and c.nenv == 12   # envs.py:69-73
    c1 = make_cn_config(clone_config(Config()), num_envs=1)
    assert c1.phase == abi.PHASE_TEST
    assert abs(c.robot_fov - 2 * 3.141592653589793) < 1e-12


def test_library_built_from_sources_on_disk(L):
    """The loaded library embeds the sha256 of the sources it was built from (build.py) and it equals
    the hash of the committed sources: GPU evidence produced with it belongs to this tree."""
    from crowdnav_dsrnn_amd import build

    ver = L.cn_version().decode()
    assert "CN_SRC_HASH=" + build.source_hash() in ver
    assert build.built_hash() == build.source_hash()
    assert not build.needs_build()
