"""ctypes front-end of the C oracle (oracle/esc_oracle.c) over packed snapshots.

TEST INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline).

``group_tables`` restates the pair numbering of include/escalator_hip.h from the group
specs (pair ids 0..n_gp-1 = distinct (label_key, label_value) in order of first
appearance), independently of the product's interner.  The C oracle then matches: a pod
is in a labelled group iff one of its pair ids is the group's (NewPodAffinityFilterFunc,
pkg/controller/node_group.go:218-253); the group named "default" takes pods through
NewPodDefaultFilterFunc instead (node_group.go:256, controller/client.go:58-64); nodes
match any group by label pair (NewNodeLabelFilterFunc node_group.go:278, :301).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("ESC_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
NONE = 0xFFFFFFFF
BRANCH_NAMES = ["empty", "gate", "below_min", "pct_err", "locked", "fast_down", "slow_down", "scale_up", "none"]
STATUS_ERR = {0: None, 1: "node count less than the minimum", 2: "node count larger than the maximum",
              3: "cannot divide by zero in percent calculation", 4: "negative scale up delta",
              5: "int64 overflow (Quantity inf.Dec regime, not emulated)"}

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.orc_totals.restype = C.c_int
        _lib.orc_totals_par.restype = C.c_int
        _lib.orc_ref_scan.restype = C.c_int
        _lib.orc_order.restype = C.c_int64
        _lib.orc_try_remove.restype = C.c_int64
        _lib.orc_percent.restype = C.c_int
        _lib.orc_scale_up.restype = C.c_int
        _lib.orc_percent.argtypes = [C.c_int64] * 5 + [C.POINTER(C.c_double)] * 2
        _lib.orc_scale_up.argtypes = [C.c_int64, C.c_double, C.c_double, C.c_int64, C.c_int64, C.c_int64,
                                      C.c_int64, C.c_int32, C.POINTER(C.c_int64)]
    return _lib


def group_tables(groups: list[dict]) -> dict:
    G = len(groups)
    default = next((i for i, g in enumerate(groups) if g["name"] == "default"), -1)
    ids: dict = {}
    gpair = np.zeros(G, np.uint32)
    for g, spec in enumerate(groups):
        k = (spec.get("label_key", ""), spec.get("label_value", ""))
        gpair[g] = ids.setdefault(k, len(ids))
    dry = np.array([1 if s.get("dry_mode") else 0 for s in groups], np.uint8)
    return {"G": G, "default": default, "gpair": gpair, "n_gp": len(ids), "pair_ids": ids, "dry": dry}


def _p(a, t):
    return np.ascontiguousarray(a).ctypes.data_as(C.POINTER(t))


def _node_args(nodes):
    return [C.c_int64(len(nodes["flags"])), _p(nodes["flags"], C.c_uint32), _p(nodes["label0"], C.c_uint32),
            _p(nodes["cpu"], C.c_int64), _p(nodes["mem"], C.c_int64)]


TOT_FIELDS = ["pod_cpu_m", "pod_mem_b", "n_pods", "node_cpu_m", "node_mem_b", "n_nodes", "n_untainted",
              "n_tainted", "n_cordoned", "first_node", "first_cpu_m", "first_mem_b", "flags"]


def totals(pods: dict, nodes: dict, groups: list[dict], node_lo: int = 0, node_hi: int | None = None,
           reference_shaped: bool = False, g_range: tuple[int, int] | None = None,
           threads: int = 0) -> np.ndarray:
    """int64 [G, 13] in esc_group_totals order.  threads > 0: orc_totals_par (OpenMP)."""
    t = group_tables(groups)
    G = t["G"]
    out = np.zeros((G, 13), np.int64)
    hi = len(nodes["flags"]) if node_hi is None else node_hi
    keep = [pods, nodes, t]
    pa = [C.c_int64(len(pods["flags"])), _p(pods["flags"], C.c_uint32), _p(pods["cpu0"], C.c_uint32),
          _p(pods["mem0"], C.c_int64), _p(pods["pair0"], C.c_uint32), _p(pods["xc_cpu"], C.c_int64),
          _p(pods["xc_mem"], C.c_int64), _p(pods["xp_pair"], C.c_uint32)]
    na = _node_args(nodes) + [_p(nodes["xl_pair"], C.c_uint32), _p(nodes["trk_node"], C.c_int32),
                              _p(nodes["trk_group"], C.c_int32), C.c_int64(len(nodes["trk_node"]))]
    if reference_shaped:
        lo, hi_g = g_range or (0, G)
        rc = lib().orc_ref_scan(*pa, *na, C.c_int32(G), C.c_int32(t["default"]), _p(t["gpair"], C.c_uint32),
                                _p(t["dry"], C.c_uint8), C.c_int32(lo), C.c_int32(hi_g), _p(out, C.c_int64))
    elif threads > 0:
        rc = lib().orc_totals_par(*pa, *na, C.c_int64(node_lo), C.c_int64(hi), C.c_int32(G),
                                  C.c_int32(t["default"]), _p(t["gpair"], C.c_uint32), C.c_uint32(t["n_gp"]),
                                  _p(t["dry"], C.c_uint8), C.c_int32(threads), _p(out, C.c_int64))
    else:
        rc = lib().orc_totals(*pa, *na, C.c_int64(node_lo), C.c_int64(hi), C.c_int32(G), C.c_int32(t["default"]),
                              _p(t["gpair"], C.c_uint32), C.c_uint32(t["n_gp"]), _p(t["dry"], C.c_uint8),
                              _p(out, C.c_int64))
    del keep
    assert rc == 0
    return out


def totals_fn(pods: dict, nodes: dict, groups: list[dict]):
    """A zero-argument callable running orc_totals (one thread) over the snapshot, its
    arguments marshalled once: the per-call CPU time of the oracle for bench.py's
    cpu_baseline figures (ctypes call overhead included, ~1 us)."""
    t = group_tables(groups)
    G = t["G"]
    out = np.zeros((G, 13), np.int64)
    arrs = {k: np.ascontiguousarray(v) for k, v in list(pods.items())}
    narrs = {k: np.ascontiguousarray(v) for k, v in list(nodes.items())}
    args = [C.c_int64(len(arrs["flags"])), _p(arrs["flags"], C.c_uint32), _p(arrs["cpu0"], C.c_uint32),
            _p(arrs["mem0"], C.c_int64), _p(arrs["pair0"], C.c_uint32), _p(arrs["xc_cpu"], C.c_int64),
            _p(arrs["xc_mem"], C.c_int64), _p(arrs["xp_pair"], C.c_uint32)]
    args += _node_args(narrs) + [_p(narrs["xl_pair"], C.c_uint32), _p(narrs["trk_node"], C.c_int32),
                                 _p(narrs["trk_group"], C.c_int32), C.c_int64(len(narrs["trk_node"]))]
    args += [C.c_int64(0), C.c_int64(len(narrs["flags"])), C.c_int32(G), C.c_int32(t["default"]),
             _p(t["gpair"], C.c_uint32), C.c_uint32(t["n_gp"]), _p(t["dry"], C.c_uint8), _p(out, C.c_int64)]
    f = lib().orc_totals
    keep = (arrs, narrs, t, out)

    def run():
        assert f(*args) == 0 and keep
        return out
    return run


def params(groups: list[dict], states: list[dict] | None) -> np.ndarray:
    out = np.zeros((len(groups), 12), np.int64)
    for g, s in enumerate(groups):
        st = (states[g] if states else None) or {}
        out[g] = [s.get("min_nodes", 0), s.get("max_nodes", 0), s.get("taint_upper_pct", 0),
                  s.get("taint_lower_pct", 0), s.get("scale_up_pct", 0), s.get("slow_removal_rate", 0),
                  s.get("fast_removal_rate", 0), int(bool(s.get("dry_mode"))), int(bool(st.get("locked", 0))),
                  st.get("requested_nodes", 0), st.get("cached_cpu_m", 0), st.get("cached_mem_b", 0)]
    return out


def decide(groups: list[dict], states: list[dict] | None, tot: np.ndarray):
    """Returns (float64 [G,2] cpu/mem pct, int64 [G,7] delta,n_to_taint,cached_cpu,cached_mem,status,branch,taint)."""
    G = len(groups)
    pr = params(groups, states)
    df = np.zeros((G, 2), np.float64)
    di = np.zeros((G, 7), np.int64)
    tot = np.ascontiguousarray(tot, np.int64)
    lib().orc_decide(C.c_int32(G), _p(pr, C.c_int64), _p(tot, C.c_int64), _p(df, C.c_double), _p(di, C.c_int64))
    return df, di


def order(nodes: dict, groups: list[dict], group: int, which: int, node_lo: int = 0,
          node_hi: int | None = None, cap: int | None = None) -> np.ndarray:
    t = group_tables(groups)
    n = len(nodes["flags"])
    hi = n if node_hi is None else node_hi
    out = np.zeros(max(hi - node_lo, 1), np.int64)
    m = lib().orc_order(C.c_int64(n), _p(nodes["flags"], C.c_uint32), _p(nodes["label0"], C.c_uint32),
                        _p(nodes["created_ns"], C.c_int64), _p(nodes["xl_pair"], C.c_uint32),
                        _p(nodes["trk_node"], C.c_int32), _p(nodes["trk_group"], C.c_int32),
                        C.c_int64(len(nodes["trk_node"])), C.c_int64(node_lo), C.c_int64(hi),
                        _p(t["dry"], C.c_uint8), _p(t["gpair"], C.c_uint32), C.c_int32(group),
                        C.c_int32(which), _p(out, C.c_int64), C.c_int64(len(out)))
    m = int(m)
    out = out[:m]
    return out if cap is None else out[:cap]


def order_all(nodes: dict, groups: list[dict], node_lo: int = 0, node_hi: int | None = None) -> dict:
    """orc_order_all: {(group, which): indices} for every group and both orders, one pass."""
    t = group_tables(groups)
    G = len(groups)
    n = len(nodes["flags"])
    hi = n if node_hi is None else node_hi
    args = [C.c_int64(n), _p(nodes["flags"], C.c_uint32), _p(nodes["label0"], C.c_uint32),
            _p(nodes["created_ns"], C.c_int64), _p(nodes["xl_pair"], C.c_uint32),
            _p(nodes["trk_node"], C.c_int32), _p(nodes["trk_group"], C.c_int32),
            C.c_int64(len(nodes["trk_node"])), C.c_int64(node_lo), C.c_int64(hi),
            _p(t["dry"], C.c_uint8), _p(t["gpair"], C.c_uint32), C.c_uint32(len(t["pair_ids"])), C.c_int32(G)]
    off = np.zeros(2 * G + 1, np.int64)
    lib().orc_order_all.restype = C.c_int64
    if lib().orc_order_all(*args, _p(off, C.c_int64), None) < 0:
        raise MemoryError("orc_order_all")
    idx = np.zeros(max(int(off[-1]), 1), np.int64)
    if lib().orc_order_all(*args, _p(off, C.c_int64), _p(idx, C.c_int64)) < 0:
        raise MemoryError("orc_order_all")
    return {(g, w): idx[off[2 * g + w]:off[2 * g + w + 1]] for g in range(G) for w in (0, 1)}


def try_remove(pods: dict, nodes: dict, groups: list[dict], pod_node, taint_s, no_delete, group: int,
               now_ns: int, soft_ns: int, hard_ns: int):
    """orc_try_remove: TryRemoveTaintedNodes for one group (scale_down.go:51-136) over a
    packed snapshot.  Returns ((n_candidates, n_delete, pods_remaining), deleted indices)."""
    t = group_tables(groups)
    n = len(nodes["flags"])
    res = np.zeros(3, np.int64)
    out = np.zeros(max(n, 1), np.int64)
    pn = np.ascontiguousarray(pod_node, np.uint32)
    ts = np.ascontiguousarray(taint_s, np.int64)
    nd = np.ascontiguousarray(no_delete, np.uint8)
    m = lib().orc_try_remove(C.c_int64(len(pods["flags"])), _p(pods["flags"], C.c_uint32),
                             _p(pods["pair0"], C.c_uint32), _p(pods["xp_pair"], C.c_uint32), _p(pn, C.c_uint32),
                             C.c_int64(n), _p(nodes["flags"], C.c_uint32), _p(nodes["label0"], C.c_uint32),
                             _p(nodes["xl_pair"], C.c_uint32), _p(nodes["trk_node"], C.c_int32),
                             _p(nodes["trk_group"], C.c_int32), C.c_int64(len(nodes["trk_node"])),
                             _p(ts, C.c_int64), _p(nd, C.c_uint8), _p(t["dry"], C.c_uint8),
                             _p(t["gpair"], C.c_uint32), C.c_int32(t["default"]), C.c_int32(group),
                             C.c_int64(now_ns), C.c_int64(soft_ns), C.c_int64(hard_ns), _p(res, C.c_int64),
                             _p(out, C.c_int64), C.c_int64(len(out)))
    if m < 0:
        raise MemoryError("orc_try_remove")
    return tuple(int(x) for x in res), out[:int(m)]


METRIC_NAMES = ["nodes", "nodes_cordoned", "nodes_untainted", "nodes_tainted", "pods", "cpu_request",
                "cpu_capacity", "mem_capacity", "mem_request", "cpu_percent", "mem_percent"]


def metrics(tot: np.ndarray, df: np.ndarray, di: np.ndarray) -> list[dict]:
    """Per-group gauges from the C oracle's totals and decisions, by the literal rules of
    oracle.node_group_metrics (controller.go:224-228, :275-278, :309-315)."""
    from oracle import oracle as O
    out = []
    for g in range(tot.shape[0]):
        t = dict(zip(TOT_FIELDS, (int(x) for x in tot[g])))
        run = {"n_nodes": t["n_nodes"], "n_cordoned": t["n_cordoned"], "n_untainted": t["n_untainted"],
               "n_tainted": t["n_tainted"], "n_pods": t["n_pods"], "pod_cpu_m": t["pod_cpu_m"],
               "pod_mem_b": t["pod_mem_b"], "node_cpu_m": t["node_cpu_m"], "node_mem_b": t["node_mem_b"],
               "branch": BRANCH_NAMES[int(di[g, 5])], "cpu_pct": float(df[g, 0]), "mem_pct": float(df[g, 1])}
        out.append(O.node_group_metrics(run))
    return out

