"""ctypes binding of the native HIP library (include/crowdnav.h).

The product path has NO fallback: if lib/libcrowdnav_hip.so is missing or fails to load, every entry
point raises. Build it with `python -m crowdnav_dsrnn_amd.build` (or __graft_entry__.build()).
"""
import ctypes
import os

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CN_LIB_PATH") or os.path.join(HERE, "lib", "libcrowdnav_hip.so")

_lib = None


class GruSeqFwd(ctypes.Structure):
    """cn_gru_seq_fwd (include/crowdnav.h): one GRU of a cn_gru_fwd_seq call (device pointers)."""
    _fields_ = [("B", ctypes.c_int64), ("gi", ctypes.c_void_p), ("w_hh", ctypes.c_void_p), ("b_hh", ctypes.c_void_p),
                ("m", ctypes.c_void_p), ("out", ctypes.c_void_p), ("hm", ctypes.c_void_p), ("save", ctypes.c_void_p),
                ("nh", ctypes.c_int64), ("x", ctypes.c_void_p), ("w_ih", ctypes.c_void_p), ("b_ih", ctypes.c_void_p),
                ("F", ctypes.c_int64)]


class GruSeqBwd(ctypes.Structure):
    """cn_gru_seq_bwd (include/crowdnav.h): one GRU of a cn_gru_bwd_seq call (device pointers)."""
    _fields_ = [("B", ctypes.c_int64), ("w_hh_t", ctypes.c_void_p), ("m", ctypes.c_void_p), ("dout", ctypes.c_void_p),
                ("save", ctypes.c_void_p), ("hm", ctypes.c_void_p), ("acc", ctypes.c_void_p), ("g", ctypes.c_void_p),
                ("db_ih", ctypes.c_void_p), ("db_hh", ctypes.c_void_p)]


class GruStepSeg(ctypes.Structure):
    """cn_gru_step_seg (include/crowdnav.h): one GRU of a cn_gru_fwd_step_group call (device pointers)."""
    _fields_ = [("B", ctypes.c_int64), ("gi", ctypes.c_void_p), ("x", ctypes.c_void_p), ("w_ih", ctypes.c_void_p),
                ("b_ih", ctypes.c_void_p), ("F", ctypes.c_int64), ("hm", ctypes.c_void_p), ("w_hh", ctypes.c_void_p),
                ("b_hh", ctypes.c_void_p), ("h_out", ctypes.c_void_p), ("h_out2", ctypes.c_void_p),
                ("g2", ctypes.c_int64), ("ld2", ctypes.c_int64)]


class NativeLibraryMissing(RuntimeError):
    pass


class StaleNativeLibrary(NativeLibraryMissing):
    """The library on disk was not built from the sources on disk (embedded CN_SRC_HASH differs)."""


def _check_provenance(L):
    """cn_version() carries the sha256 of the sources the library was built from (build.py). When the
    sources are present (always in-tree, on the GPU box too) they must hash to the same value."""
    from . import build

    ver = L.cn_version().decode()
    mark = build.HASH_MARK.decode()
    got = ver.split(mark, 1)[1][:64] if mark in ver else None
    if os.environ.get("CN_LIB_PATH") or not all(os.path.exists(d) for d in build.DEPS):
        return ver
    want = build.source_hash()
    if got != want:
        raise StaleNativeLibrary(
            "%s was built from other sources (embedded %s, sources on disk %s): rebuild with "
            "`python -m crowdnav_dsrnn_amd.build`" % (LIB_PATH, got, want))
    return ver


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeLibraryMissing(
            "HIP engine library not built: %s is missing (run `python -m crowdnav_dsrnn_amd.build`)" % LIB_PATH)
    # torch's HIP runtime first: the library's libamdhip64 dependency then binds to the runtime torch already
    # loaded (torch ships its own copy). Loaded the other way round, the process holds two HIP runtimes, the
    # streams and device pointers the host side passes in belong to the other one, and the library's first
    # launch fails with hipErrorNoDevice.
    import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    cfgp = ctypes.POINTER(abi.CnConfig)
    L.cn_last_error.restype = ctypes.c_char_p
    L.cn_version.restype = ctypes.c_char_p
    _check_provenance(L)
    L.cn_config_validate.argtypes = [cfgp]
    L.cn_create.argtypes = [cfgp, ctypes.c_int, ctypes.POINTER(vp)]
    L.cn_create_mixed.argtypes = [cfgp, ctypes.c_int, vp, i64, ctypes.c_int, ctypes.POINTER(vp)]
    L.cn_env_humans.argtypes = [vp, vp]
    L.cn_destroy.argtypes = [vp]
    L.cn_destroy.restype = None
    L.cn_reset.argtypes = [vp, vp, vp, vp, vp]
    L.cn_step.argtypes = [vp, vp, vp] + [vp] * 9
    L.cn_step_seq.argtypes = [vp, vp, ctypes.c_int, vp, i64] + [vp] * 9
    L.cn_state_bytes.argtypes = [vp, ctypes.POINTER(i64)]
    L.cn_state_layout_offsets.argtypes = [cfgp, ctypes.POINTER(i64), ctypes.POINTER(i64)]
    L.cn_state_field_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_int),
                                      ctypes.POINTER(ctypes.c_int)]
    L.cn_get_state.argtypes = [vp, vp, vp, ctypes.c_int]
    L.cn_set_state.argtypes = [vp, vp, vp, ctypes.c_int]
    L.cn_state_device_ptr.argtypes = [vp]
    L.cn_state_device_ptr.restype = vp
    L.cn_edge_features.argtypes = [vp, i64, ctypes.c_int] + [vp] * 14
    L.cn_gru_fwd_step.argtypes = [vp, i64, ctypes.c_int] + [vp] * 7
    L.cn_gru_fwd_step_scatter.argtypes = [vp, i64, ctypes.c_int] + [vp] * 8 + [i64, i64]
    L.cn_gru_fwd_fused.argtypes = [vp, i64, ctypes.c_int] + [vp] * 9 + [i64, i64]
    L.cn_debug_disc_quad.argtypes = [vp, i64, ctypes.c_int] + [vp] * 6
    L.cn_debug_orca.argtypes = [vp, i64, ctypes.c_int, vp, vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp]
    L.cn_debug_copy64.argtypes = [vp, i64, ctypes.c_int, vp, vp]
    L.cn_orca_predict.argtypes = [vp, i64, ctypes.c_int, vp, vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp]
    L.cn_orca_predict_kd.argtypes = [vp, i64, ctypes.c_int, vp, vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp,
                                     vp]
    L.cn_debug_set_spawn_budget.argtypes = [vp, ctypes.c_longlong]
    L.cn_debug_spawn_stats.argtypes = [vp, vp]
    L.cn_social_force_predict.argtypes = [vp, i64, ctypes.c_int, vp, vp] + [ctypes.c_double] * 4 + [vp]
    L.cn_gru_bwd_step.argtypes = [vp, i64, ctypes.c_int] + [vp] * 7
    L.cn_lidar_obs.argtypes = [vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double, vp, vp]
    L.cn_attn_pool_fwd.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int] + [vp] * 3
    L.cn_attn_pool_bwd.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int] + [vp] * 5
    try:
        L.cn_gru_bias_blocks.argtypes = [i64]
        L.cn_gru_bias_blocks.restype = i64
        L.cn_gru_bias_work_elems.argtypes = [ctypes.c_int]
        L.cn_gru_bias_work_elems.restype = i64
        L.cn_gru_bwd_step_bias.argtypes = [vp, i64, ctypes.c_int] + [vp] * 8
        L.cn_gru_bwd_step_bias.restype = i32
        L.cn_gru_bwd_step_gates.argtypes = [vp, i64, ctypes.c_int] + [vp] * 7
        L.cn_gru_bwd_step_gates.restype = i32
        L.cn_gru_bias_reduce.argtypes = [vp, i64, ctypes.c_int] + [vp] * 4
        L.cn_gru_bias_reduce.restype = i32
        L.cn_gae.argtypes = [vp, ctypes.c_int, i64, ctypes.c_float, ctypes.c_float, ctypes.c_int] + [vp] * 5
        L.cn_gae.restype = i32
        L.cn_gaussian_act.argtypes = [vp, i64, ctypes.c_int] + [vp] * 5
        L.cn_gaussian_act.restype = i32
        L.cn_gru_bwd_seq_work_elems.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(GruSeqBwd)]
        L.cn_gru_bwd_seq_work_elems.restype = i64
        L.cn_gru_fwd_step_group.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(GruStepSeg)]
        L.cn_gru_fwd_step_group.restype = i32
        L.cn_gru_fwd_seq.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(GruSeqFwd)]
        L.cn_gru_fwd_seq.restype = i32
        L.cn_gru_bwd_seq.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(GruSeqBwd), vp, i64]
        L.cn_gru_bwd_seq.restype = i32
        L.cn_set_graph_mode.argtypes = [vp, vp, ctypes.c_int]
        L.cn_graph_node_counts.argtypes = [vp, ctypes.POINTER(i64), ctypes.c_int, ctypes.POINTER(i64)]
        L.cn_graph_node_counts.restype = i32
        L.cn_wgrad_work_elems.argtypes = [i64, ctypes.c_int, ctypes.c_int]
        L.cn_wgrad_work_elems.restype = i64
        L.cn_wgrad.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int] + [vp] * 6
        L.cn_spatial_attn_fwd.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int, ctypes.c_float] + [vp] * 5
        L.cn_spatial_attn_bwd.argtypes = [vp, i64, ctypes.c_int, ctypes.c_int, ctypes.c_float] + [vp] * 7 + [i64, vp, i64]
    except AttributeError:
        if not os.environ.get("CN_LIB_PATH"):   # an older diagnostic library (A/B runs) may lack them
            raise
    L.cn_profile.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    L.cn_profile_read.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(i64)]
    for f in ("cn_config_validate", "cn_create", "cn_create_mixed", "cn_env_humans", "cn_reset", "cn_step", "cn_step_seq", "cn_state_bytes", "cn_state_layout_offsets",
              "cn_state_field_info", "cn_get_state", "cn_set_state", "cn_edge_features", "cn_profile",
              "cn_profile_read", "cn_gru_fwd_step", "cn_gru_fwd_step_scatter", "cn_gru_fwd_fused", "cn_gru_bwd_step", "cn_attn_pool_fwd", "cn_attn_pool_bwd", "cn_spatial_attn_fwd", "cn_spatial_attn_bwd", "cn_wgrad", "cn_set_graph_mode", "cn_lidar_obs", "cn_debug_disc_quad", "cn_debug_orca", "cn_debug_copy64", "cn_orca_predict", "cn_orca_predict_kd", "cn_social_force_predict", "cn_debug_set_spawn_budget", "cn_debug_spawn_stats"):
        if hasattr(L, f) or not os.environ.get("CN_LIB_PATH"):
            getattr(L, f).restype = i32
    _lib = L
    return L


GRAPH_NODE_TYPES = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event", "event_record",
                    "ext_sem_signal", "ext_sem_wait", "mem_alloc", "mem_free", "memcpy_from_symbol",
                    "memcpy_to_symbol")


def graph_node_counts(graph):
    """{node type: count} of a captured hipGraph_t (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()),
    through cn_graph_node_counts; types with no node are left out. 'total' = all nodes."""
    n = len(GRAPH_NODE_TYPES)
    counts = (ctypes.c_int64 * n)()
    total = ctypes.c_int64()
    check(lib().cn_graph_node_counts(ctypes.c_void_p(graph), counts, n, ctypes.byref(total)))
    out = {GRAPH_NODE_TYPES[k]: int(counts[k]) for k in range(n) if counts[k]}
    out["total"] = int(total.value)
    return out


def check(rc):
    if rc != 0:
        raise RuntimeError("crowdnav native error %d: %s" % (rc, lib().cn_last_error().decode()))
    return rc


EXPORTED = ["cn_last_error", "cn_version", "cn_config_validate", "cn_create", "cn_create_mixed", "cn_env_humans",
            "cn_destroy", "cn_reset", "cn_step", "cn_step_seq",
            "cn_state_bytes", "cn_state_layout_offsets", "cn_state_field_info", "cn_get_state", "cn_set_state",
            "cn_state_device_ptr", "cn_edge_features", "cn_profile", "cn_profile_read", "cn_gru_fwd_step", "cn_gru_fwd_step_scatter",
            "cn_gru_fwd_fused", "cn_gru_bwd_step", "cn_attn_pool_fwd", "cn_attn_pool_bwd", "cn_spatial_attn_fwd",
            "cn_spatial_attn_bwd", "cn_wgrad_work_elems", "cn_wgrad",
            "cn_gru_bias_blocks", "cn_gru_bwd_step_bias", "cn_gru_bwd_step_gates", "cn_gru_bias_work_elems", "cn_gru_bias_reduce",
            "cn_gru_bwd_seq_work_elems", "cn_gru_fwd_step_group", "cn_gru_fwd_seq", "cn_gru_bwd_seq", "cn_gaussian_act", "cn_gae",
            "cn_set_graph_mode", "cn_graph_node_counts", "cn_lidar_obs", "cn_debug_disc_quad",
            "cn_debug_orca", "cn_debug_copy64", "cn_orca_predict", "cn_orca_predict_kd", "cn_social_force_predict",
            "cn_debug_set_spawn_budget", "cn_debug_spawn_stats"]
