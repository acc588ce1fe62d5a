"""Marshalling of pod / node records into the C ABI's object structs.

A pod or node is a plain dict carrying exactly the ``v1.Pod`` / ``v1.Node`` fields the
hot path reads (what the cgo shim copies out of the Go objects):

pod:  {"name", "owner_kinds": [str], "annotations": {str: str},
       "node_selector": {k: v} | None,
       "affinity": None | {"node_affinity": None | {"required": None | [[{"key", "op", "values"}]]},
                           "pod_affinity": bool, "pod_anti_affinity": bool},
       "containers": [{"cpu": int|None, "mem": int|None}], "init_containers": [...],
       "overhead": None | {"cpu": int|None, "mem": int|None}, "node_name": str}
node: {"name", "labels": {k: v}, "unschedulable": bool, "taints": [key], "cpu": int|None,
       "mem": int|None, "created_ns": int}

Quantities are already MilliValue() (cpu) / Value() (memory) integers; ``None`` is an
absent resource key.
"""
from __future__ import annotations

import ctypes as C
import re

from . import _lib as L


def _b(s) -> bytes:
    return (s if s is not None else "").encode()


class _Keep:
    """Owns every ctypes buffer referenced by a marshalled batch."""

    def __init__(self):
        self.refs = []

    def arr(self, ctype, items):
        a = (ctype * max(len(items), 1))(*items)
        self.refs.append(a)
        return a

    def cstrs(self, strs):
        bs = [_b(s) for s in strs]
        self.refs.append(bs)
        return self.arr(C.c_char_p, bs)


def _req(r) -> L.Request:
    if r is None:
        return L.Request(0, 0, 0, 0)
    cpu, mem = r.get("cpu"), r.get("mem")
    return L.Request(cpu or 0, mem or 0, int(cpu is not None), int(mem is not None))


def pods_to_c(pods: list[dict]):
    keep = _Keep()
    out = (L.PodObj * max(len(pods), 1))()
    for i, p in enumerate(pods):
        o = out[i]
        kinds = list(p.get("owner_kinds") or [])
        o.owner_kinds = keep.cstrs(kinds)
        o.n_owner_kinds = len(kinds)
        ann = p.get("annotations") or {}
        if "kubernetes.io/config.source" in ann:
            o.has_config_source = 1
            v = _b(ann["kubernetes.io/config.source"])
            keep.refs.append(v)
            o.config_source = v
        sel = p.get("node_selector") or {}
        kvs = []
        for k, v in sel.items():
            kb, vb = _b(k), _b(v)
            keep.refs.extend([kb, vb])
            kvs.append(L.KV(kb, vb))
        o.node_selector = keep.arr(L.KV, kvs)
        o.n_node_selector = len(kvs)
        aff = p.get("affinity")
        exprs = []
        if aff is not None:
            o.has_affinity = 1
            na = aff.get("node_affinity")
            o.has_pod_affinity = int(bool(aff.get("pod_affinity")))
            o.has_pod_anti_affinity = int(bool(aff.get("pod_anti_affinity")))
            if na is not None:
                o.has_node_affinity = 1
                req = na.get("required")
                if req is not None:
                    o.has_required = 1
                    for t, term in enumerate(req):
                        for e in term:
                            vals = list(e.get("values") or [])
                            kb, ob = _b(e["key"]), _b(e["op"])
                            keep.refs.extend([kb, ob])
                            exprs.append(L.SelectorExpr(kb, ob, keep.cstrs(vals), len(vals), t))
        o.exprs = keep.arr(L.SelectorExpr, exprs)
        o.n_exprs = len(exprs)
        cs = [_req(c) for c in p.get("containers") or []]
        o.containers = keep.arr(L.Request, cs)
        o.n_containers = len(cs)
        ic = [_req(c) for c in p.get("init_containers") or []]
        o.init_containers = keep.arr(L.Request, ic)
        o.n_init_containers = len(ic)
        ovh = p.get("overhead")
        if ovh is not None:
            o.has_overhead = 1
            o.overhead = _req(ovh)
    keep.refs.append(out)
    return out, len(pods), keep


def nodes_to_c(nodes: list[dict]):
    keep = _Keep()
    out = (L.NodeObj * max(len(nodes), 1))()
    for i, n in enumerate(nodes):
        o = out[i]
        nb = _b(n.get("name"))
        keep.refs.append(nb)
        o.name = nb
        kvs = []
        for k, v in (n.get("labels") or {}).items():
            kb, vb = _b(k), _b(v)
            keep.refs.extend([kb, vb])
            kvs.append(L.KV(kb, vb))
        o.labels = keep.arr(L.KV, kvs)
        o.n_labels = len(kvs)
        o.unschedulable = int(bool(n.get("unschedulable")))
        taints = list(n.get("taints") or [])
        o.taint_keys = keep.cstrs(taints)
        o.n_taints = len(taints)
        o.allocatable = _req({"cpu": n.get("cpu"), "mem": n.get("mem")})
        o.created_unix_ns = int(n.get("created_ns", 0))
    keep.refs.append(out)
    return out, len(nodes), keep


def groups_to_c(groups: list[dict]):
    keep = _Keep()
    out = (L.GroupSpec * len(groups))()
    for i, g in enumerate(groups):
        o = out[i]
        for f in ("name", "label_key", "label_value"):
            b = _b(g.get(f, ""))
            keep.refs.append(b)
            setattr(o, f, b)
        o.min_nodes = g.get("min_nodes", 0)
        o.max_nodes = g.get("max_nodes", 0)
        o.taint_upper_pct = g.get("taint_upper_pct", 0)
        o.taint_lower_pct = g.get("taint_lower_pct", 0)
        o.scale_up_pct = g.get("scale_up_pct", 0)
        o.slow_removal_rate = g.get("slow_removal_rate", 0)
        o.fast_removal_rate = g.get("fast_removal_rate", 0)
        o.dry_mode = int(bool(g.get("dry_mode", False)))
    keep.refs.append(out)
    return out, keep


def groups_from_c(specs, n: int) -> list[dict]:
    out = []
    for i in range(n):
        s = specs[i]
        out.append({"name": s.name.decode(), "label_key": s.label_key.decode(),
                    "label_value": s.label_value.decode(), "min_nodes": s.min_nodes,
                    "max_nodes": s.max_nodes, "taint_upper_pct": s.taint_upper_pct,
                    "taint_lower_pct": s.taint_lower_pct, "scale_up_pct": s.scale_up_pct,
                    "slow_removal_rate": s.slow_removal_rate, "fast_removal_rate": s.fast_removal_rate,
                    "dry_mode": bool(s.dry_mode)})
    return out


def states_to_c(states: list[dict] | None, n: int):
    out = (L.GroupState * n)()
    for i in range(n):
        st = (states[i] if states else None) or {}
        out[i] = L.GroupState(int(bool(st.get("locked", 0))), st.get("requested_nodes", 0),
                              st.get("cached_cpu_m", 0), st.get("cached_mem_b", 0))
    return out


# ------------------------------------------------ scale-down reaping inputs (§8f rank 2)
TO_BE_REMOVED_KEY = "atlassian.com/escalator"          # pkg/k8s/taint.go:31 (ToBeRemovedByAutoscalerKey)
NO_DELETE_ANNOTATION = "atlassian.com/no-delete"       # pkg/controller/scale_down.go:22
INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1
_NONE = 0xFFFFFFFF


def taint_time(node: dict) -> int:
    """GetToBeRemovedTime (pkg/k8s/taint.go:91-103) as Unix seconds: INT64_MIN when the
    escalator taint is absent or its value is not a base-10 int64 (strconv.ParseInt)."""
    if TO_BE_REMOVED_KEY not in (node.get("taints") or []):
        return INT64_MIN
    v = node.get("taint_value")
    if not isinstance(v, str) or not re.fullmatch(r"[+-]?[0-9]+", v):
        return INT64_MIN
    t = int(v)
    # INT64_MIN itself doubles as "no time": the one parseable value treated as absent
    return t if INT64_MIN < t <= INT64_MAX else INT64_MIN


def placement(pods: list[dict], nodes: list[dict]):
    """Inputs of esc_load_placement from objects, in the packer's pod / node order:
    each pod's Spec.NodeName as a node index (NONE when empty or not a listed node:
    CreateNodeNameToInfoMap drops those, node_state.go:31-36), each node's escalator-taint
    time and its no-delete annotation (safeFromDeletion, scale_down.go:39-46)."""
    import numpy as np
    # CreateNodeNameToInfoMap is keyed by name: two nodes sharing one would share one
    # NodeInfo (node_state.go:10-39).  Kubernetes node names are unique, so a duplicate is
    # an input error here rather than a pod run silently attached to one of them.
    index = {}
    for j, n in enumerate(nodes):
        name = n.get("name", "")
        if name in index:
            raise ValueError("duplicate node name %r (nodes %d and %d)" % (name, index[name], j))
        index[name] = j
    pod_node = np.array([index.get(p.get("node_name") or "", _NONE) if p.get("node_name") else _NONE
                         for p in pods], np.uint32)
    taint_s = np.array([taint_time(n) for n in nodes], np.int64)
    no_delete = np.array([1 if (n.get("annotations") or {}).get(NO_DELETE_ANNOTATION, "") else 0 for n in nodes],
                         np.uint8)
    return pod_node, taint_s, no_delete
