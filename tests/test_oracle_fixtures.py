"""Pin the CPU oracle to the reference's own known-answer tests (tests/golden/*.json)."""
import struct

import pytest

from builders import build_test_node, build_test_nodes, build_test_pod, build_test_pods, unix_ns
from oracle import oracle as O


def _pods(fx, names):
    return [build_test_pod(fx["pods"][n]) for n in names]


def test_pod_is_daemonset(golden):
    for c in golden["k8s_util"]["pod_is_daemonset"]:
        assert O.pod_is_daemonset(build_test_pod(c["pod"])) is c["want"], c["src"]


def test_pod_is_static(golden):
    for c in golden["k8s_util"]["pod_is_static"]:
        assert O.pod_is_static(build_test_pod(c["pod"])) is c["want"], c["src"]


def test_calculate_pods_requests_total(golden):
    fx = golden["k8s_util"]
    for c in fx["calculate_pods_requests_total"]:
        mem, cpu = O.calculate_pods_requests_total(_pods(fx, c["pods"]))
        assert (mem, cpu) == (c["mem"], c["cpu"]), c["name"]


def test_calculate_nodes_capacity_total(golden):
    fx = golden["k8s_util"]
    for c in fx["calculate_nodes_capacity_total"]:
        nodes = [build_test_node(fx["nodes"][n]) for n in c["nodes"]]
        mem, cpu = O.calculate_nodes_capacity_total(nodes)
        assert (mem, cpu) == (c["mem"], c["cpu"]), c["name"]


def test_calc_percent_usage(golden):
    for c in golden["controller"]["calc_percent_usage"]:
        cpu, mem, err = O.calc_percent_usage(*c["args"])
        assert cpu == c["cpu"] and mem == c["mem"] and err == c["err"], c["name"]


def test_calc_scale_up_delta_below_threshold(golden):
    """Property of util_test.go:15-192."""
    for c in golden["controller"]["calc_scale_up_delta_below_threshold"]["cases"]:
        n_p, p_cpu, p_mem = c["pods"]
        n_n, n_cpu, n_mem = c["nodes"]
        pods = build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]})
        nodes = build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem})
        mem_r, cpu_r = O.calculate_pods_requests_total(pods)
        mem_c, cpu_c = O.calculate_nodes_capacity_total(nodes)
        cpu_p, mem_p, _ = O.calc_percent_usage(cpu_r, mem_r, cpu_c, mem_c, len(nodes))
        want, _ = O.calc_scale_up_delta(len(nodes), cpu_p, mem_p, cpu_r, mem_r, 0, 0, c["threshold"])
        if want <= 0:
            continue
        nodes2 = nodes + build_test_nodes(want, {"CPU": n_cpu, "Mem": n_mem}, "m")
        mem_c, cpu_c = O.calculate_nodes_capacity_total(nodes2)
        cpu2, mem2, _ = O.calc_percent_usage(cpu_r, mem_r, cpu_c, mem_c, len(nodes2))
        assert cpu2 <= c["threshold"] and mem2 <= c["threshold"], c


def test_filters(golden):
    fx = golden["controller"]
    for c in fx["pod_affinity_filter"]["cases"]:
        pod = build_test_pod(fx["pod_affinity_filter"]["pods"][c["pod"]])
        assert O.new_pod_affinity_filter_func(c["key"], c["value"])(pod) is c["want"], c["name"]
    for c in fx["pod_default_filter"]["cases"]:
        pod = build_test_pod(fx["pod_default_filter"]["pods"][c["pod"]])
        assert O.new_pod_default_filter_func()(pod) is c["want"], c["name"]
    for c in fx["node_label_filter"]["cases"]:
        node = build_test_node(fx["node_label_filter"]["nodes"][c["node"]])
        assert O.new_node_label_filter_func(c["key"], c["value"])(node) is c["want"], c["name"]


def test_sorts(golden):
    fx = golden["controller"]
    old = [unix_ns(*d) for d in fx["sort_dates"]["oldest_ordered"]]
    new = [unix_ns(*d) for d in fx["sort_dates"]["newest_ordered"]]
    # 1 ns apart entries (sort_test.go:28-31) must order strictly
    assert old[4] - old[3] == 1
    import random
    rng = random.Random(7)
    for _ in range(20):
        perm = list(range(6))
        rng.shuffle(perm)
        shuffled = [old[i] for i in perm]
        assert [perm[i] for i in O.oldest_first(shuffled)] == list(range(6))
        shuffled = [new[i] for i in perm]
        assert [perm[i] for i in O.newest_first(shuffled)] == list(range(6))
    dates = [unix_ns(*d) for d in fx["six_nodes"]["dates"]]
    for c in fx["taint_oldest_n"]:
        assert O.taint_oldest_n(dates[:c["slice"]], c["n"]) == c["want"], c["name"]
    for c in fx["untaint_newest_n"]:
        assert O.untaint_newest_n(dates[:c["slice"]], c["n"]) == c["want"], c["name"]
    for c in fx["scale_down_taint"]:
        n, err = O.scale_down_taint_clamp(c["untainted"], c["n"], c["min"])
        assert (n if err is None else 0, err) == (c["want"], c["err"]), c["name"]


def test_filter_nodes(golden):
    fx = golden["controller"]["filter_nodes"]
    nodes = [build_test_node(o) for o in fx["nodes"]]
    for c in fx["cases"]:
        assert O.filter_nodes(c["dry"], c["tracker"], nodes) == (c["untainted"], c["tainted"], c["cordoned"])


def _default_group(opts):
    g = {"name": "default", "label_key": "", "label_value": ""}
    g.update(opts)
    g.setdefault("max_nodes", 0)
    return g


def test_scale_node_group(golden):
    for c in golden["controller"]["scale_node_group"]["cases"]:
        if c.get("lister_error"):
            continue        # lister failures are host-side; tests/test_host_api.py covers them
        n_n, n_cpu, n_mem = c["nodes"]
        n_p, p_cpu, p_mem = c["pods"]
        nodes = build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem})
        pods = build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]})
        g = _default_group(c["opts"])
        out = O.scale_node_group(g, {}, pods, nodes)
        assert out["delta"] == c["delta"] and out["err"] == c["err"], (c["name"], out)
        if out["delta"] > 0:
            nodes2 = nodes + build_test_nodes(out["delta"], {"CPU": n_cpu, "Mem": n_mem}, "m")
            st = {"cached_cpu_m": out["cached_cpu_m"], "cached_mem_b": out["cached_mem_b"]}
            assert O.scale_node_group(g, st, pods, nodes2)["delta"] == 0, c["name"]


def test_scale_node_group_multiple_runs_first(golden):
    for c in golden["controller"]["scale_node_group_multiple_runs"]["cases"]:
        n_n, n_cpu, n_mem = c["nodes"]
        n_p, p_cpu, p_mem = c["pods"]
        nodes = build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem})
        pods = build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]})
        st = {}
        if c["cached"]:
            st = {"cached_cpu_m": c["cached"][0], "cached_mem_b": c["cached"][1]}
        out = O.scale_node_group(_default_group(c["opts"]), st, pods, nodes)
        assert out["delta"] == c["delta"] and out["err"] is None, (c["name"], out)


def test_untaint_min_max(golden):
    for c in golden["controller"]["untaint_min_max_nodes"]["cases"]:
        nodes = build_test_nodes(c["tainted"][0], {"CPU": c["tainted"][1], "Mem": c["tainted"][2], "Tainted": True}, "t")
        nodes += build_test_nodes(c["untainted"][0], {"CPU": c["untainted"][1], "Mem": c["untainted"][2]}, "u")
        pods = build_test_pods(c["pods"][0], {"CPU": [c["pods"][1]], "Mem": [c["pods"][2]]})
        out = O.scale_node_group(_default_group(c["opts"]), {}, pods, nodes)
        assert out["branch"] == c["branch"] and out["delta"] == c["delta"], (c["name"], out)
        # ScaleUp untaints newest-first over the tainted list; all of them here
        assert len(out["tainted"]) <= out["delta"]


def test_known_float_bits():
    """SURVEY.md §8c re-derived vectors: cpu% = 333.33333333333337 (0x1.4d55555555556p+8)."""
    cpu, mem, _ = O.calc_percent_usage(100 * 500, 100 * 600, 10 * 1500, 10 * 5000, 10)
    assert struct.pack("<d", cpu) == struct.pack("<d", float.fromhex("0x1.4d55555555556p+8"))
    assert mem == 120.0


def test_go_semantics_edges():
    assert O._go_int(float("nan")) == O.INT64_MIN
    assert O._go_int(float("inf")) == O.INT64_MIN
    assert O._go_max(float("nan"), float("inf")) == float("inf")
    assert O.milli_value_mem((1 << 62)) == O.wrap64((1 << 62) * 1000)
    # threshold 0 (bypassed validation): (cpu-0)/0 = +Inf -> int(Inf) -> negative delta error
    d, err = O.calc_scale_up_delta(3, 50.0, 50.0, 1, 1, 1, 1, 0)
    assert d == O.INT64_MIN and err == O.ERR_NEG_DELTA
    with pytest.raises(O.QuantityOverflow):
        O.quantity_add(O.INT64_MAX, 1)


def test_metrics_gauges_follow_scale_node_group_returns(golden):
    """node_group_metrics: which gauges each return path of scaleNodeGroup Sets
    (controller.go:224-228 always; :275-278 after the min/max gates; :309-315 after a
    successful calcPercentUsage) on the reference's TestScaleNodeGroup cases.  The gauge
    values themselves are not asserted by any reference test (parity unpinned beyond the
    restatement)."""
    always = {"nodes", "nodes_cordoned", "nodes_untainted", "nodes_tainted", "pods"}
    req = {"cpu_request", "cpu_capacity", "mem_capacity", "mem_request"}
    pct = {"cpu_percent", "mem_percent"}
    seen = set()
    for c in golden["controller"]["scale_node_group"]["cases"]:
        if c.get("lister_error"):
            continue
        n_n, n_cpu, n_mem = c["nodes"]
        n_p, p_cpu, p_mem = c["pods"]
        out = O.scale_node_group(_default_group(c["opts"]), {}, build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]}),
                                 build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem}))
        m = O.node_group_metrics(out)
        want = always | (req if out["branch"] not in ("empty", "gate") else set()) | \
            (pct if out["branch"] not in ("empty", "gate", "below_min", "pct_err") else set())
        assert set(m) == want, (c["name"], out["branch"], sorted(m))
        assert m["nodes"] == float(n_n)
        if "cpu_percent" in m and out["cpu_pct"] != O.MAX_FLOAT64:
            assert m["cpu_percent"] == out["cpu_pct"]
        seen.add(out["branch"])
    assert len(seen) >= 3


def test_metrics_memory_gauge_quirk():
    """float64(mem.MilliValue() / 1000): the ×1000 product wraps in int64 before Go's
    truncating division (unpinned; restated from apimachinery v0.22.5)."""
    out = {"n_nodes": 1, "n_cordoned": 0, "n_untainted": 1, "n_tainted": 0, "n_pods": 1, "pod_cpu_m": 5,
           "pod_mem_b": 1 << 62, "node_cpu_m": 7, "node_mem_b": 3, "branch": "none", "cpu_pct": 1.0, "mem_pct": 2.0}
    m = O.node_group_metrics(out)
    assert m["mem_capacity"] == 3.0
    assert m["mem_request"] == float(O.go_div_trunc(O.wrap64((1 << 62) * 1000), 1000))
    assert O.go_div_trunc(-1999, 1000) == -1 and O.go_div_trunc(1999, -1000) == -1


# ------------------------------------------- §8f rank 2: node_state.go / TryRemoveTaintedNodes
def _ns_golden():
    import json
    import os
    return json.load(open(os.path.join(os.path.dirname(__file__), "golden", "node_state.json")))


def test_create_node_name_to_info_map_fixtures():
    for c in _ns_golden()["create_node_name_to_info_map"]:
        nodes = [{"name": n} for n in c["nodes"]]
        pods = [{"node_name": n, "owner_kinds": []} for n in c["pods"]]
        m = O.create_node_name_to_info_map(pods, nodes)
        assert len(m) == c["want_len"], c["name"]
        assert sum(len(v["pods"]) for v in m.values()) == c["want_pods"], c["name"]


def test_node_empty_and_pods_remaining_fixtures():
    for c in _ns_golden()["node_state"]:
        node = {"name": "node-1"}
        pods = [{"node_name": "node-1", "owner_kinds": [p["owner"]] if p["owner"] else []} for p in c["pods"]]
        m = None if c["empty_map"] else O.create_node_name_to_info_map(pods, [node])
        assert O.node_empty(node, m) == c["empty"], c["name"]
        assert O.node_pods_remaining(node, m) == (c["remaining"], c["ok"]), c["name"]


def test_try_remove_tainted_nodes_fixtures():
    g = _ns_golden()["try_remove_tainted_nodes"]
    now_s = 1_700_000_000
    for c in g["cases"]:
        nodes = [{"name": "n%d" % i, "taints": ["atlassian.com/escalator"], "taint_value": str(now_s),
                  "created_ns": i} for i in range(10)]
        pods = [{"node_name": "", "owner_kinds": []} for _ in range(10)]
        tainted = nodes[:c["n_tainted"]]
        if c["annotate_first_tainted"]:
            tainted[0]["annotations"] = {"atlassian.com/no-delete": "skip for testing"}
        got, _, _ = O.try_remove_tainted_nodes({"name": "default"}, tainted, pods, nodes,
                                                now_ns=now_s * 1_000_000_000 + 1, soft_ns=0, hard_ns=0,
                                                dry_mode=False)
        assert got == c["want"], c["name"]


def test_to_be_removed_time_parse():
    """strconv.ParseInt(v, 10, 64) semantics for the taint value (taint.go:95)."""
    t = {"taints": ["atlassian.com/escalator"]}
    assert O.get_to_be_removed_time(dict(t, taint_value="1700000000")) == 1700000000
    assert O.get_to_be_removed_time(dict(t, taint_value="+12")) == 12
    for bad in ("", " 12", "1_000", "12s", "9223372036854775808", None):
        assert O.get_to_be_removed_time(dict(t, taint_value=bad)) is None, bad
    assert O.get_to_be_removed_time({"taints": [], "taint_value": "12"}) is None
