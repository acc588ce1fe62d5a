"""ctypes binding of libescalator_hip.so (the C ABI in include/escalator_hip.h).

The shared library is built in-tree (``escalator_amd/libescalator_hip.so``) by
``__graft_entry__.build()`` / ``make -C escalator_amd/csrc``.  Loading fails loudly when
it is missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ESC_LIB_PATH: an alternative build of the same library (the host-sanitizer build of
# scripts/asan_check.sh); the default is the in-tree gfx950 build.
LIB_PATH = os.environ.get("ESC_LIB_PATH") or os.path.join(HERE, "libescalator_hip.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "escalator_hip.h")

ESC_OK = 0
ESC_E_INVAL, ESC_E_HIP, ESC_E_NOMEM, ESC_E_LIMIT, ESC_E_STATE, ESC_E_NODEV, ESC_E_COMM = -1, -2, -3, -4, -5, -6, -7
ESC_E_ORDER = -8                    # a K5 ordering's bounded look-back gave up (that ordering only)
ESC_COMM_ID_BYTES = 128
ESC_SEL_NONE, ESC_SEL_TAINT, ESC_SEL_UNTAINT, ESC_SEL_CUT = -1, 0, 1, 4
ESC_NONE = 0xFFFFFFFF

ESC_ST_OK, ESC_ST_ERR_MIN_NODES, ESC_ST_ERR_MAX_NODES, ESC_ST_ERR_DIV_ZERO = 0, 1, 2, 3
ESC_ST_ERR_NEG_DELTA, ESC_ST_ERR_OVERFLOW, ESC_ST_ERR_TAINT_MIN = 4, 5, 6
ESC_ST_NOT_OWNED = 7                # world > 1: decided on the group's owner rank
ESC_TF_NOT_OWNED = 4
BRANCHES = ["empty", "gate", "below_min", "pct_err", "locked", "fast_down", "slow_down", "scale_up", "none"]

PF_DAEMONSET, PF_STATIC, PF_HAS_SEL, PF_AFF_BLOCK, PF_HAS_OVH = 1, 2, 4, 8, 16
PF_XREG_SHIFT, PF_XINIT_SHIFT, PF_XPAIR_SHIFT = 8, 16, 24
NF_UNSCHED, NF_TAINTED, NF_TRACKED, NF_XLBL_SHIFT = 1, 2, 4, 8
TF_POD_OVERFLOW, TF_NODE_OVERFLOW = 1, 2

i32, i64, u32, u64, dbl = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64, C.c_double
cstr = C.c_char_p
P = C.POINTER


class GroupSpec(C.Structure):
    _fields_ = [("name", cstr), ("label_key", cstr), ("label_value", cstr),
                ("min_nodes", i32), ("max_nodes", i32), ("taint_upper_pct", i32),
                ("taint_lower_pct", i32), ("scale_up_pct", i32), ("slow_removal_rate", i32),
                ("fast_removal_rate", i32), ("dry_mode", i32)]


class GroupState(C.Structure):
    _fields_ = [("locked", i32), ("requested_nodes", i32), ("cached_cpu_m", i64), ("cached_mem_b", i64)]


class GroupTotals(C.Structure):
    _fields_ = [(n, i64) for n in ("pod_cpu_m", "pod_mem_b", "n_pods", "node_cpu_m", "node_mem_b",
                                   "n_nodes", "n_untainted", "n_tainted", "n_cordoned", "first_node",
                                   "first_cpu_m", "first_mem_b", "flags")]


class GroupDecision(C.Structure):
    _fields_ = [("cpu_pct", dbl), ("mem_pct", dbl), ("delta", i64), ("n_to_taint", i64),
                ("cached_cpu_m", i64), ("cached_mem_b", i64), ("status", i32), ("branch", i32),
                ("taint_status", i32), ("reserved", i32)]


class GroupMetrics(C.Structure):
    _fields_ = [(n, dbl) for n in ("nodes", "nodes_cordoned", "nodes_untainted", "nodes_tainted", "pods",
                                   "cpu_request", "cpu_capacity", "mem_capacity", "mem_request",
                                   "cpu_percent", "mem_percent")] + [("set_mask", u32), ("reserved", u32)]


METRIC_NAMES = [n for n, _ in GroupMetrics._fields_[:11]]


class Removal(C.Structure):
    _fields_ = [("n_candidates", i64), ("n_delete", i64), ("pods_remaining", i64), ("reserved", i64)]


class KV(C.Structure):
    _fields_ = [("key", cstr), ("value", cstr)]


class Request(C.Structure):
    _fields_ = [("cpu_m", i64), ("mem_b", i64), ("has_cpu", i32), ("has_mem", i32)]


class SelectorExpr(C.Structure):
    _fields_ = [("key", cstr), ("op", cstr), ("values", P(cstr)), ("n_values", i32), ("term", i32)]


class PodObj(C.Structure):
    _fields_ = [("owner_kinds", P(cstr)), ("n_owner_kinds", i32), ("has_config_source", i32),
                ("config_source", cstr), ("node_selector", P(KV)), ("n_node_selector", i32),
                ("has_affinity", i32), ("has_node_affinity", i32), ("has_pod_affinity", i32),
                ("has_pod_anti_affinity", i32), ("has_required", i32), ("exprs", P(SelectorExpr)),
                ("n_exprs", i32), ("containers", P(Request)), ("n_containers", i32),
                ("init_containers", P(Request)), ("n_init_containers", i32), ("has_overhead", i32),
                ("overhead", Request)]


class NodeObj(C.Structure):
    _fields_ = [("name", cstr), ("labels", P(KV)), ("n_labels", i32), ("unschedulable", i32),
                ("taint_keys", P(cstr)), ("n_taints", i32), ("allocatable", Request),
                ("created_unix_ns", i64)]


class PodSoA(C.Structure):
    _fields_ = [("n_pods", i64), ("flags", P(u32)), ("cpu0", P(u32)), ("mem0", P(i64)),
                ("pair0", P(u32)), ("xc_cpu", P(i64)), ("xc_mem", P(i64)), ("n_xc", i64),
                ("xp_pair", P(u32)), ("n_xp", i64)]


class NodeSoA(C.Structure):
    _fields_ = [("n_nodes", i64), ("flags", P(u32)), ("label0", P(u32)), ("cpu", P(i64)),
                ("mem", P(i64)), ("created_ns", P(i64)), ("xl_pair", P(u32)), ("n_xl", i64),
                ("trk_node", P(i32)), ("trk_group", P(i32)), ("n_trk", i64)]


class SynthParams(C.Structure):
    _fields_ = [("n_pods", i64), ("n_nodes", i64), ("n_groups", i32), ("config", i32),
                ("seed", u64), ("with_default", i32), ("n_threads", i32)]


VP = C.c_void_p
_SIGS = {
    "esc_abi_version": (i32, []),
    "esc_strerror": (cstr, [i32]),
    "esc_status_string": (cstr, [i32]),
    "esc_taint_error": (i32, [i64, i32, C.c_char_p, i32]),
    "esc_ctx_create": (i32, [P(GroupSpec), i32, i32, i32, i32, P(VP)]),
    "esc_ctx_create_multi": (i32, [P(GroupSpec), i32, P(i32), i32, P(VP)]),
    "esc_ctx_counts": (i32, [VP, P(i64), P(i64)]),
    "esc_group_owner": (i32, [VP, i32, P(i32)]),
    "esc_node_owner_ranges": (i32, [VP, P(NodeSoA), i32, P(u32)]),
    "esc_exchange_rows": (i32, [VP, P(NodeSoA), i32, P(u32), P(i32)]),
    "esc_comm_size": (i32, [VP, P(i32)]),
    "esc_ctx_destroy": (i32, [VP]),
    "esc_ctx_set_stream": (i32, [VP, VP]),
    "esc_ctx_num_groups": (i32, [VP]),
    "esc_ctx_pair_id": (u32, [VP, cstr, cstr]),
    "esc_ctx_num_group_pairs": (i32, [VP]),
    "esc_packer_create": (i32, [VP, P(VP)]),
    "esc_packer_destroy": (i32, [VP]),
    "esc_packer_add_pods": (i32, [VP, P(PodObj), i64]),
    "esc_packer_add_nodes": (i32, [VP, P(NodeObj), i64]),
    "esc_packer_set_tracker": (i32, [VP, i32, P(cstr), i64]),
    "esc_packer_set_list_mode": (i32, [VP, i32]),
    "esc_packer_view": (i32, [VP, P(PodSoA), P(NodeSoA)]),
    "esc_load_pods": (i32, [VP, P(PodSoA), i64]),
    "esc_load_nodes": (i32, [VP, P(NodeSoA), i64, i64]),
    "esc_set_replicas": (i32, [VP, i32]),
    "esc_stream_bytes": (i32, [VP, P(i64), P(i64)]),
    "esc_set_state": (i32, [VP, P(GroupState)]),
    "esc_reduce": (i32, [VP]),
    "esc_exchange_buffers": (i32, [VP, P(VP), P(i64), P(VP), P(i64)]),
    "esc_exchange_slice": (i32, [VP, P(i64), P(i64)]),
    "esc_bind_exchange_buffers": (i32, [VP, VP, VP]),
    "esc_exchange_download": (i32, [VP, P(i64), P(i64)]),
    "esc_exchange_upload": (i32, [VP, P(i64), P(i64)]),
    "esc_decide": (i32, [VP]),
    "esc_run": (i32, [VP]),
    "esc_sync": (i32, [VP]),
    "esc_comm_unique_id": (i32, [VP]),
    "esc_comm_init": (i32, [VP, VP, i32, i32]),
    "esc_exchange": (i32, [VP]),
    "esc_step": (i32, [VP]),
    "esc_results": (i32, [VP, P(GroupTotals), P(GroupDecision)]),
    "esc_set_spare": (i32, [VP, dbl]),
    "esc_pods_upsert": (i32, [VP, P(i64), P(PodSoA)]),
    "esc_pods_delete": (i32, [VP, P(i64), i64]),
    "esc_nodes_update": (i32, [VP, P(i64), i64, P(u32), P(i64), P(i64)]),
    "esc_nodes_add": (i32, [VP, P(NodeSoA), P(i64)]),
    "esc_nodes_delete": (i32, [VP, P(i64), i64]),
    "esc_nodes_relabel": (i32, [VP, P(i64), P(NodeSoA)]),
    "esc_hbm_probe": (i32, [VP, i64, i32, P(C.c_double)]),
    "esc_tracker_update": (i32, [VP, i32, P(i64), i64, P(i64), i64]),
    "esc_tracker_list": (i32, [VP, i32, P(i64), i64, P(i64)]),
    "esc_load_placement": (i32, [VP, P(u32), P(i64), P(C.c_uint8)]),
    "esc_try_remove": (i32, [VP, i64, P(i64), P(i64), P(Removal)]),
    "esc_pods_bind": (i32, [VP, P(i64), P(u32), i64]),
    "esc_reap_occupancy": (i32, [VP]),
    "esc_reap_buffer": (i32, [VP, P(VP), P(i64)]),
    "esc_reap_download": (i32, [VP, P(u32)]),
    "esc_reap_upload": (i32, [VP, P(u32)]),
    "esc_reap_finish": (i32, [VP, i64, P(i64), P(i64), P(Removal)]),
    "esc_removal_nodes": (i32, [VP, i32, P(i64), i64, P(i64)]),
    "esc_set_metrics": (i32, [VP, i32]),
    "esc_metrics_results": (i32, [VP, P(GroupMetrics)]),
    "esc_use_graph": (i32, [VP, i32]),
    "esc_force_wide": (i32, [VP, i32]),
    "esc_set_timing": (i32, [VP, i32]),
    "esc_stage_times": (i32, [VP, P(dbl), i32]),
    "esc_k1_trace": (i32, [VP, P(C.c_uint64), i64, P(i64)]),
    "esc_k1_calibrate": (i32, [VP, i32]),
    "esc_k1_time": (i32, [VP, i32, P(C.c_double)]),
    "esc_k1_flush_entries": (i32, [VP, P(i64), P(i64)]),
    "esc_sort_nodes": (i32, [VP]),
    "esc_set_order_in_step": (i32, [VP, i32]),
    "esc_build_age_index": (i32, [VP]),
    "esc_order_info": (i32, [VP, P(i64), P(i32)]),
    "esc_group_order": (i32, [VP, i32, i32, P(i64), i64, P(i64)]),
    "esc_set_selections": (i32, [VP, i32, i32]),
    "esc_selections": (i32, [VP, P(i32), P(i64), P(i64), i64, P(i64)]),
    "esc_pods_requests_total": (i32, [VP, P(PodObj), i64, P(i64), P(i64)]),
    "esc_nodes_capacity_total": (i32, [VP, P(NodeObj), i64, P(i64), P(i64)]),
    "esc_order_by_creation": (i32, [VP, P(i64), i64, i32, i64, P(i64)]),
    "esc_calc_percent_usage": (i32, [i64, i64, i64, i64, i64, P(dbl), P(dbl)]),
    "esc_calc_scale_up_delta": (i32, [i64, dbl, dbl, i64, i64, i64, i64, i32, P(i64)]),
    "esc_synth_create": (i32, [P(SynthParams), i64, i64, P(VP)]),
    "esc_synth_destroy": (i32, [VP]),
    "esc_synth_groups": (i32, [VP, P(P(GroupSpec)), P(i32)]),
    "esc_synth_states": (i32, [VP, P(P(GroupState))]),
    "esc_synth_view": (i32, [VP, P(PodSoA), P(NodeSoA)]),
    "esc_synth_objects": (i32, [VP, P(P(PodObj)), P(i64), P(P(NodeObj)), P(i64)]),
}

_lib = None


class EscError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = load().esc_strerror(code).decode() if _lib is not None else str(code)
        super().__init__("%s: %s (%d)" % (what, msg, code) if what else "%s (%d)" % (msg, code))


def load():
    """Load the in-tree HIP library; raise if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("escalator_amd: %s is missing — run __graft_entry__.build() "
                              "(make -C escalator_amd/csrc); there is no CPU fallback" % LIB_PATH)
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64, so when torch
        # is installed it is loaded first and the library binds to that runtime (loading
        # /opt/rocm's first and torch's second leaves two runtimes that disagree on devices).
        if not os.environ.get("ESC_NO_TORCH_PRELOAD"):   # sanitizer runs keep torch out
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != ESC_OK:
        raise EscError(rc, what)


def header_functions() -> list[str]:
    """Every function the C header declares (used by the ABI export test)."""
    import re
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(esc_[a-z_0-9]+)\s*\(", txt, flags=re.M)))
