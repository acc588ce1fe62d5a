"""CPU oracle — literal restatement of Escalator's scale-decision hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``escalator_amd``) may import,
call or link this module: only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg use it, and only as the checker.

Parity status: PINNED by the reference's own known-answer tests, transcribed as data
into ``tests/golden/*.json`` (``tests/test_oracle_fixtures.py`` checks this module
against every one of them).  The reference is Go; no Go toolchain or k8s module cache
exists in this image, so the reference itself cannot be run and no
``oracle/_ref`` build exists.

Third-party semantics restated here (not vendored in /root/reference):
``k8s.io/apimachinery v0.22.5`` ``pkg/api/resource`` (go.mod:15) — ``Quantity.Add``,
``MilliValue``, ``Value``, ``IsZero`` on int64 amounts.  Restated from the published
algorithm: int64 amounts add with an overflow check (overflow switches the Quantity
to an ``inf.Dec`` — reported here as ``OverflowError``-style status, not emulated);
``MilliValue()`` of a scale-0 amount multiplies by 1000 and keeps the wrapped int64
product (parity unpinned: no reference test reaches it).

Objects are plain dicts mirroring the ``v1.Pod`` / ``v1.Node`` fields the path reads
(schema in ``escalator_amd/objects.py``; builders in ``tests/builders.py``).
Go semantics reproduced exactly: int64 two's-complement wrap for ``Resource`` sums,
IEEE-754 float64 for the percentages (Python floats are binary64; int->float is
round-half-even like Go's conversion), ``math.Ceil``/``math.Max`` special cases and
amd64's ``int(float64)`` conversion of NaN/Inf (0x8000000000000000).
"""
from __future__ import annotations

import re

import math

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1
MAX_FLOAT64 = 1.7976931348623157e308          # math.MaxFloat64

DEFAULT_NODE_GROUP = "default"                # pkg/controller/node_group.go:16
TO_BE_REMOVED_KEY = "atlassian.com/escalator" # pkg/k8s/taint.go:31

ERR_MIN_NODES = "node count less than the minimum"                    # controller.go:239
ERR_MAX_NODES = "node count larger than the maximum"                  # controller.go:248
ERR_DIV_ZERO = "cannot divide by zero in percent calculation"         # util.go:75
ERR_NEG_DELTA = "negative scale up delta"                             # util.go:43
ERR_OVERFLOW = "int64 overflow (Quantity inf.Dec regime, not emulated)"


def wrap64(x: int) -> int:
    """Go int64 two's-complement wrap."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


class QuantityOverflow(Exception):
    """Quantity.Add left int64 (the reference would continue in inf.Dec)."""


def quantity_add(a: int, b: int) -> int:
    """apimachinery Quantity.Add on two int64 amounts of one scale (checked add)."""
    s = a + b
    if s < INT64_MIN or s > INT64_MAX:
        raise QuantityOverflow()
    return s


def milli_value_mem(b: int) -> int:
    """Quantity.MilliValue() of a scale-0 memory amount: value*1000, wrapped (unpinned)."""
    return wrap64(b * 1000)


# ---------------------------------------------------------------- pkg/k8s/util.go
def pod_is_daemonset(pod: dict) -> bool:
    """PodIsDaemonSet — pkg/k8s/util.go:11-18: any OwnerReferences[].Kind == "DaemonSet"."""
    return any(k == "DaemonSet" for k in pod.get("owner_kinds") or [])


def pod_is_static(pod: dict) -> bool:
    """PodIsStatic — pkg/k8s/util.go:21-24."""
    ann = pod.get("annotations") or {}
    return "kubernetes.io/config.source" in ann and ann["kubernetes.io/config.source"] == "file"


def compute_pod_resource_request(pod: dict) -> tuple[int, int]:
    """ComputePodResourceRequest — pkg/k8s/scheduler/types.go:72-89.

    Resource.Add (:14-27) sums present keys with plain int64 += (wraps);
    SetMaxResource (:30-43) takes max only over present keys; Overhead is added only
    when Spec.Overhead != nil (:84).  Returns (milli_cpu, memory)."""
    cpu = 0
    mem = 0
    for c in pod.get("containers") or []:
        if c.get("cpu") is not None:
            cpu = wrap64(cpu + c["cpu"])
        if c.get("mem") is not None:
            mem = wrap64(mem + c["mem"])
    for c in pod.get("init_containers") or []:
        if c.get("mem") is not None:
            mem = mem if mem >= c["mem"] else c["mem"]          # types.go:89, max :91
        if c.get("cpu") is not None:
            cpu = cpu if cpu >= c["cpu"] else c["cpu"]
    ovh = pod.get("overhead")
    if ovh is not None:
        if ovh.get("cpu") is not None:
            cpu = wrap64(cpu + ovh["cpu"])
        if ovh.get("mem") is not None:
            mem = wrap64(mem + ovh["mem"])
    return cpu, mem


def calculate_pods_requests_total(pods: list[dict]) -> tuple[int, int]:
    """CalculatePodsRequestsTotal — pkg/k8s/util.go:27-38.  Returns (mem, cpu)."""
    mem = 0
    cpu = 0
    for p in pods:
        c, m = compute_pod_resource_request(p)
        mem = quantity_add(mem, m)
        cpu = quantity_add(cpu, c)
    return mem, cpu


def node_alloc(node: dict) -> tuple[int, int]:
    """Allocatable.Cpu().MilliValue(), Allocatable.Memory().Value(); absent -> zero Quantity."""
    c = node.get("cpu")
    m = node.get("mem")
    return (0 if c is None else c), (0 if m is None else m)


def calculate_nodes_capacity_total(nodes: list[dict]) -> tuple[int, int]:
    """CalculateNodesCapacityTotal — pkg/k8s/util.go:41-51.  Returns (mem, cpu)."""
    mem = 0
    cpu = 0
    for n in nodes:
        c, m = node_alloc(n)
        mem = quantity_add(mem, m)
        cpu = quantity_add(cpu, c)
    return mem, cpu


# ------------------------------------------------- pkg/controller/node_group.go
def unwrap_node_selector_terms(pod: dict):
    """unwrapNodeSelectorTerms — node_group.go:208-215."""
    aff = pod.get("affinity")
    if aff is not None and aff.get("node_affinity") is not None:
        req = aff["node_affinity"].get("required")
        if req is not None:
            return req
    return None


def new_pod_affinity_filter_func(label_key: str, label_value: str):
    """NewPodAffinityFilterFunc — node_group.go:218-253."""
    def f(pod: dict) -> bool:
        if pod_is_daemonset(pod):
            return False
        sel = pod.get("node_selector")
        if sel is not None and label_key in sel and sel[label_key] == label_value:
            return True
        for term in unwrap_node_selector_terms(pod) or []:
            for expr in term:
                if expr["key"] != label_key:
                    continue
                if expr["op"] == "In":
                    for v in expr.get("values") or []:
                        if v == label_value:
                            return True
        return False
    return f


def new_pod_default_filter_func():
    """NewPodDefaultFilterFunc — node_group.go:256-275."""
    def f(pod: dict) -> bool:
        if pod_is_daemonset(pod):
            return False
        if pod_is_static(pod):
            return False
        aff = pod.get("affinity")
        return len(pod.get("node_selector") or {}) == 0 and (
            aff is None or (aff.get("node_affinity") is None and not aff.get("pod_affinity")
                            and not aff.get("pod_anti_affinity")))
    return f


def new_node_label_filter_func(label_key: str, label_value: str):
    """NewNodeLabelFilterFunc — node_group.go:278-287."""
    def f(node: dict) -> bool:
        labels = node.get("labels") or {}
        return label_key in labels and labels[label_key] == label_value
    return f


def group_pod_filter(group: dict):
    """pkg/controller/client.go:58-64: "default" -> default filter, else affinity filter."""
    if group["name"] == DEFAULT_NODE_GROUP:
        return new_pod_default_filter_func()
    return new_pod_affinity_filter_func(group.get("label_key", ""), group.get("label_value", ""))


def filtered_list(items: list, pred) -> list:
    """FilteredPodsLister.List / FilteredNodesLister.List — pkg/k8s/pod_listers.go:33,
    node_listers.go:33: order-preserving filter of the full list."""
    return [x for x in items if pred(x)]


# --------------------------------------------- pkg/controller/controller.go
def has_to_be_removed_taint(node: dict) -> bool:
    """GetToBeRemovedTaint — pkg/k8s/taint.go:80-87."""
    return any(k == TO_BE_REMOVED_KEY for k in node.get("taints") or [])


def filter_nodes(dry_mode: bool, tracker: list[str], all_nodes: list[dict]):
    """(*Controller).filterNodes — controller.go:120-154.  Returns index lists
    (untainted, tainted, cordoned) into all_nodes."""
    unt, tnt, cor = [], [], []
    for i, node in enumerate(all_nodes):
        if dry_mode:
            if node.get("name") in tracker:
                tnt.append(i)
            else:
                unt.append(i)
        else:
            if node.get("unschedulable"):
                cor.append(i)
                continue
            if has_to_be_removed_taint(node):
                tnt.append(i)
            else:
                unt.append(i)
    return unt, tnt, cor


# ------------------------------------------------ pkg/k8s/node_state.go + taint.go:91
def create_node_name_to_info_map(pods: list[dict], nodes: list[dict]) -> dict:
    """CreateNodeNameToInfoMap — node_state.go:10-39: pods grouped by Spec.NodeName, then
    node infos without a node ("" or unknown names: pods out of sync) removed."""
    m: dict = {}
    for p in pods:
        m.setdefault(p.get("node_name", ""), {"node": None, "pods": []})["pods"].append(p)
    for n in nodes:
        m.setdefault(n["name"], {"node": None, "pods": []})["node"] = n
    return {k: v for k, v in m.items() if v["node"] is not None}


def node_pods_remaining(node: dict, info_map: dict | None) -> tuple[int, bool]:
    """NodePodsRemaining — node_state.go:48-65: non-daemonset pods on the node, ok = the
    node is in the map."""
    if not info_map or node["name"] not in info_map:
        return 0, False
    return sum(1 for p in info_map[node["name"]]["pods"] if not pod_is_daemonset(p)), True


def node_empty(node: dict, info_map: dict | None) -> bool:
    """NodeEmpty — node_state.go:42-45."""
    n, ok = node_pods_remaining(node, info_map)
    return ok and n == 0


def get_to_be_removed_time(node: dict):
    """GetToBeRemovedTime — taint.go:91-103: the escalator taint's value as Unix seconds;
    None when the taint is absent or its value does not parse (strconv.ParseInt)."""
    if not has_to_be_removed_taint(node):
        return None
    v = node.get("taint_value")
    if not isinstance(v, str) or not re.fullmatch(r"[+-]?[0-9]+", v):   # strconv.ParseInt(v, 10, 64)
        return None
    t = int(v)
    return t if INT64_MIN <= t <= INT64_MAX else None


def try_remove_tainted_nodes(group: dict, tainted: list[dict], pods_g: list[dict], all_nodes: list[dict],
                             now_ns: int, soft_ns: int, hard_ns: int, dry_mode: bool) -> tuple[int, int, list[int]]:
    """(*Controller).TryRemoveTaintedNodes — scale_down.go:51-136 (the cloud-provider and
    API deletes stay with the host).  Returns (-len(toBeDeleted), podsRemaining summed over
    them, indices into `tainted` of the nodes to delete)."""
    info = create_node_name_to_info_map(pods_g, all_nodes)          # controller.go:259
    out = []
    for k, node in enumerate(tainted):
        ann = node.get("annotations") or {}
        if ann.get("atlassian.com/no-delete", ""):                   # safeFromDeletion :39-46
            continue
        t = get_to_be_removed_time(node)
        if t is None:                                                # :65-69
            continue
        age = now_ns - t * 1_000_000_000                             # now.Sub(taintedTime)
        if age > soft_ns:
            if node_empty(node, info) or age > hard_ns:
                if not dry_mode:
                    out.append(k)
    remaining = 0
    for k in out:
        n, ok = node_pods_remaining(tainted[k], info)
        if ok:
            remaining += n
    return -len(out), remaining, out


# ------------------------------------------------ pkg/controller/util.go
def _go_max(x: float, y: float) -> float:
    """math.Max special cases (Go stdlib)."""
    if math.isinf(x) and x > 0 or math.isinf(y) and y > 0:
        return math.inf
    if math.isnan(x) or math.isnan(y):
        return math.nan
    if x == 0 and y == 0:
        return y if math.copysign(1.0, x) < 0 else x
    return x if x > y else y


def _fdiv(a: float, b: float) -> float:
    """IEEE-754 binary64 division (Python raises on /0; Go and the GPU do not)."""
    if b == 0.0:
        if a == 0.0 or math.isnan(a):
            return math.nan
        return math.copysign(math.inf, a) * math.copysign(1.0, b)
    return a / b


def _go_ceil(x: float) -> float:
    if math.isnan(x) or math.isinf(x):
        return x
    return float(math.ceil(x))


def _go_int(x: float) -> int:
    """int(float64) on amd64 (CVTTSD2SQ): NaN/Inf/out-of-range -> INT64_MIN."""
    if math.isnan(x) or math.isinf(x) or x >= 9.223372036854775808e18 or x < -9.223372036854775808e18:
        return INT64_MIN
    return int(x)   # truncation toward zero


def calc_percent_usage(cpu_req_m: int, mem_req_b: int, cpu_cap_m: int, mem_cap_b: int,
                       n_untainted: int):
    """calcPercentUsage — pkg/controller/util.go:58-81.  Returns (cpu, mem, err)."""
    a, b, c, d = cpu_req_m, milli_value_mem(mem_req_b), cpu_cap_m, milli_value_mem(mem_cap_b)
    if a == 0 and b == 0 and c == 0 and d == 0 and n_untainted == 0:   # allEqual :48
        return 0.0, 0.0, None
    if c == 0 or d == 0:
        if n_untainted == 0:
            return MAX_FLOAT64, MAX_FLOAT64, None
        return 0.0, 0.0, ERR_DIV_ZERO
    cpu = _fdiv(float(a), float(c)) * 100.0
    mem = _fdiv(float(b), float(d)) * 100.0
    return cpu, mem, None


def calc_scale_up_delta(n_untainted: int, cpu_pct: float, mem_pct: float, cpu_req_m: int,
                        mem_req_b: int, cached_cpu_m: int, cached_mem_b: int,
                        scale_up_pct: int):
    """calcScaleUpDelta — pkg/controller/util.go:13-46.  Returns (delta, err)."""
    node_count = float(n_untainted)
    t = float(scale_up_pct)
    if cpu_pct == MAX_FLOAT64 or mem_pct == MAX_FLOAT64:
        if cached_cpu_m == 0 or cached_mem_b == 0:          # Quantity.IsZero
            return 1, None
        need_cpu = _go_ceil(_fdiv(_fdiv(float(cpu_req_m), float(cached_cpu_m)), t) * 100.0)
        need_mem = _go_ceil(_fdiv(_fdiv(float(milli_value_mem(mem_req_b)),
                                        float(milli_value_mem(cached_mem_b))), t) * 100.0)
    else:
        pc = _fdiv(cpu_pct - t, t)
        pm = _fdiv(mem_pct - t, t)
        need_cpu = _go_ceil(node_count * pc)
        need_mem = _go_ceil(node_count * pm)
    delta = _go_int(_go_max(need_cpu, need_mem))
    if delta < 0:
        return delta, ERR_NEG_DELTA
    return delta, None


# ------------------------------------------ scale_down.go / scale_up.go / sort.go
def scale_down_taint_clamp(n_untainted: int, nodes_delta: int, min_nodes: int):
    """scaleDownTaint clamp — pkg/controller/scale_down.go:138-158.  Returns (n, err)."""
    n = nodes_delta
    if n_untainted - n < min_nodes:
        n = n_untainted - min_nodes
        if n < 0:
            return 0, ("the number of nodes(%d) is less than specified minimum of %d. "
                       "Taking no action" % (n_untainted, min_nodes))
    return n, None


def oldest_first(created_ns: list[int]) -> list[int]:
    """sort.Sort(nodesByOldestCreationTime) — sort.go:18-20 (Before = strict <).
    Ties are unordered in Go; here they keep input order (stable)."""
    return sorted(range(len(created_ns)), key=lambda i: created_ns[i])


def newest_first(created_ns: list[int]) -> list[int]:
    """sort.Sort(nodesByNewestCreationTime) — sort.go:33-35."""
    return sorted(range(len(created_ns)), key=lambda i: -created_ns[i])


def taint_oldest_n(created_ns: list[int], n: int) -> list[int]:
    """taintOldestN — scale_down.go:171-205, dry mode (every taint succeeds)."""
    return oldest_first(created_ns)[:max(n, 0)]


def untaint_newest_n(created_ns: list[int], n: int) -> list[int]:
    """untaintNewestN — scale_up.go:118-163 over the tainted list (every untaint succeeds)."""
    return newest_first(created_ns)[:max(n, 0)]


# ------------------------------------------------------ scaleNodeGroup (pure part)
def go_div_trunc(a: int, b: int) -> int:
    """Go's int64 '/' (truncates toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def node_group_metrics(out: dict) -> dict:
    """The gauges scaleNodeGroup Sets in the run that produced `out` (pkg/metrics/metrics.go):
    controller.go:224-228 before any gate; :275-278 after the min/max gates
    (float64(cpu.MilliValue()), float64(mem.MilliValue() / 1000)); :309-315 after a
    successful calcPercentUsage (0 when scaling up from 0).  Absent key = not Set."""
    m = {"nodes": float(out["n_nodes"]), "nodes_cordoned": float(out["n_cordoned"]),
         "nodes_untainted": float(out["n_untainted"]), "nodes_tainted": float(out["n_tainted"]),
         "pods": float(out["n_pods"])}
    if out["branch"] in ("empty", "gate"):
        return m
    m["cpu_request"] = float(out["pod_cpu_m"])
    m["cpu_capacity"] = float(out["node_cpu_m"])
    m["mem_capacity"] = float(go_div_trunc(milli_value_mem(out["node_mem_b"]), 1000))
    m["mem_request"] = float(go_div_trunc(milli_value_mem(out["pod_mem_b"]), 1000))
    if out["branch"] in ("below_min", "pct_err"):
        return m
    from_zero = out["cpu_pct"] == MAX_FLOAT64 or out["mem_pct"] == MAX_FLOAT64
    m["cpu_percent"] = 0.0 if from_zero else out["cpu_pct"]
    m["mem_percent"] = 0.0 if from_zero else out["mem_pct"]
    return m


def scale_node_group(group: dict, state: dict, pods: list[dict], nodes: list[dict],
                     global_dry_mode: bool = False, tracker: list[str] | None = None) -> dict:
    """(*Controller).scaleNodeGroup — controller.go:192-397, decision arithmetic only.

    `pods`/`nodes` are the full cluster lists in lister order; the group's listers
    filter them (node_group.go:290-303).  Actuation (ScaleUp/ScaleDown API calls,
    controller.go:367-383) is outside the hot path: the returned dict carries the delta
    and the ordering inputs the actuation would consume."""
    pods_g = filtered_list(pods, group_pod_filter(group))
    nodes_idx = [i for i, n in enumerate(nodes)
                 if new_node_label_filter_func(group.get("label_key", ""),
                                               group.get("label_value", ""))(n)]
    all_nodes = [nodes[i] for i in nodes_idx]
    cached_cpu = state.get("cached_cpu_m", 0)
    cached_mem = state.get("cached_mem_b", 0)
    if all_nodes:                                                    # :208-211
        cached_cpu, cached_mem = node_alloc(all_nodes[0])
    dry = bool(global_dry_mode or group.get("dry_mode"))
    unt, tnt, cor = filter_nodes(dry, tracker or [], all_nodes)      # :214
    out = dict(n_pods=len(pods_g), n_nodes=len(all_nodes), n_untainted=len(unt),
               n_tainted=len(tnt), n_cordoned=len(cor), cached_cpu_m=cached_cpu,
               cached_mem_b=cached_mem, cpu_pct=0.0, mem_pct=0.0, delta=0, err=None,
               branch="none", n_to_taint=0, taint_err=None,
               first_node=(nodes_idx[0] if nodes_idx else -1),
               untainted=[nodes_idx[i] for i in unt], tainted=[nodes_idx[i] for i in tnt])
    min_nodes = group.get("min_nodes", 0)
    max_nodes = group.get("max_nodes", 0)
    try:
        mem_req, cpu_req = calculate_pods_requests_total(pods_g)
        mem_cap, cpu_cap = calculate_nodes_capacity_total([all_nodes[i] for i in unt])
    except QuantityOverflow:
        mem_req = cpu_req = mem_cap = cpu_cap = None
    out.update(pod_cpu_m=cpu_req, pod_mem_b=mem_req, node_cpu_m=cpu_cap, node_mem_b=mem_cap)
    if not all_nodes and not pods_g:                                 # :233
        out["branch"] = "empty"
        return out
    if len(all_nodes) < min_nodes:                                   # :238
        out.update(branch="gate", err=ERR_MIN_NODES)
        return out
    if len(all_nodes) > max_nodes:                                   # :247
        out.update(branch="gate", err=ERR_MAX_NODES)
        return out
    if cpu_req is None:
        out.update(branch="gate", err=ERR_OVERFLOW)
        return out
    if len(unt) < min_nodes:                                         # :281
        out.update(branch="below_min", delta=min_nodes - len(unt))
        return out
    cpu_pct, mem_pct, err = calc_percent_usage(cpu_req, mem_req, cpu_cap, mem_cap, len(unt))
    out.update(cpu_pct=cpu_pct, mem_pct=mem_pct)
    if err is not None:                                              # :300
        out.update(branch="pct_err", err=err, cpu_pct=cpu_pct, mem_pct=mem_pct)
        return out
    if state.get("locked"):                                          # :317
        out.update(branch="locked", delta=state.get("requested_nodes", 0))
        return out
    max_pct = _go_max(cpu_pct, mem_pct)                              # :328
    if max_pct < float(group.get("taint_lower_pct", 0)):
        out.update(branch="fast_down", delta=-group.get("fast_removal_rate", 0))
    elif max_pct < float(group.get("taint_upper_pct", 0)):
        out.update(branch="slow_down", delta=-group.get("slow_removal_rate", 0))
    elif max_pct > float(group.get("scale_up_pct", 0)):
        delta, err = calc_scale_up_delta(len(unt), cpu_pct, mem_pct, cpu_req, mem_req,
                                         cached_cpu, cached_mem, group.get("scale_up_pct", 0))
        out.update(branch="scale_up", delta=delta, err=err)
        if err is not None:
            return out
    if out["delta"] < 0:                                             # :368 -> ScaleDown
        n, terr = scale_down_taint_clamp(len(unt), -out["delta"], min_nodes)
        out.update(n_to_taint=n, taint_err=terr)
    return out
