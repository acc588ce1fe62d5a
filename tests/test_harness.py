"""The cgo shim's call sequence, run by the plain-C harness (go/escalatorhip/harness) on
random object clusters.  Without a device the harness must stop at the first device call
with ESC_E_NODEV after the host-side calls (packer, scalar math) succeeded; on the GPU its
totals, decisions, status strings and orderings must equal the literal oracle's."""
import random
import struct

import pytest

import harness_io as H
from oracle import oracle as O
from randobj import make_groups, make_nodes, make_pods, make_states, make_trackers


def _cluster(seed: int):
    rng = random.Random(7100 + seed)
    G = rng.choice([1, 4, 9])
    groups = make_groups(rng, G, with_default=rng.random() < 0.6)
    pods = make_pods(rng, rng.choice([0, 40, 300]) if seed else 0, groups, big_frac=0.02)
    nodes = make_nodes(rng, rng.choice([5, 30, 120]) if seed else 0, groups, big_frac=0.0)
    trackers = make_trackers(rng, groups, nodes)
    return groups, make_states(rng, G), pods, nodes, trackers


@pytest.fixture(scope="module")
def harness():
    return H.build_harness()


def test_harness_host_only_stops_at_device_call(harness, tmp_path):
    groups, states, pods, nodes, trackers = _cluster(3)
    path = str(tmp_path / "in.txt")
    H.write_input(path, groups, states, pods, nodes, trackers, device=-1)
    r = H.run(path)
    assert r["nodev"] == "esc_load_pods"
    assert int(r["abi"][0]) >= 3
    # host-only scalar math: calcPercentUsage(20000m, 40000B, 20000m, 80000B) = 100 %, 50 %
    st, cpu, mem = r["pct"]
    assert int(st) == 0
    assert struct.unpack("<d", bytes.fromhex(cpu)[::-1])[0] == 100.0
    assert struct.unpack("<d", bytes.fromhex(mem)[::-1])[0] == 50.0
    cpu_pct, mem_pct, err = O.calc_percent_usage(20000, 40000, 20000, 80000, 10)
    d, derr = O.calc_scale_up_delta(10, cpu_pct, mem_pct, 20000, 40000, 0, 0, 70)
    assert r["delta"] == ["0", str(d)] and derr is None
    assert int(r["packed"][0]) == len(pods) and int(r["packed"][3]) == len(nodes)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,shards", [(s, 0) for s in range(6)] + [(1, 1), (2, 2), (5, 3)])
def test_harness_shim_sequence_vs_literal(harness, tmp_path, seed, shards):
    """seed 0 is the empty cluster (every array NULL); shards > 0 runs the NewContextMulti
    sequence (one context over `shards` copies of device 0)."""
    from escalator_amd._lib import BRANCHES
    groups, states, pods, nodes, trackers = _cluster(seed)
    path = str(tmp_path / "in.txt")
    H.write_input(path, groups, states, pods, nodes, trackers, device=0)
    r = H.run(path, shards=shards)
    assert r["nodev"] is None and r["lines"].rstrip().endswith("done")
    for g, spec in enumerate(groups):
        L = O.scale_node_group(spec, states[g], pods, nodes, tracker=trackers.get(g, []))
        t, d = r["totals"][g], r["decision"][g]
        assert t[2] == L["n_pods"] and t[5:10] == [L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"],
                                                   L["first_node"]], g
        if L["pod_cpu_m"] is not None:
            assert [t[0], t[1], t[3], t[4]] == [L["pod_cpu_m"], L["pod_mem_b"], L["node_cpu_m"], L["node_mem_b"]], g
        assert BRANCHES[d["branch"]] == L["branch"], (g, L)
        assert d["delta"] == L["delta"] and d["n_to_taint"] == L["n_to_taint"], (g, L)
        assert d["cpu_bits"] == struct.unpack("<Q", struct.pack("<d", L["cpu_pct"]))[0]
        assert d["mem_bits"] == struct.unpack("<Q", struct.pack("<d", L["mem_pct"]))[0]
        assert (d["cached_cpu_m"], d["cached_mem_b"]) == (L["cached_cpu_m"], L["cached_mem_b"])
        err, terr = r["status"][g].split("|")
        assert err == (L["err"] or ""), g
        assert terr == (L["taint_err"] or ""), g
        unt, tn = L["untainted"], L["tainted"]
        oldest = [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
        newest = [tn[i] for i in O.newest_first([nodes[i]["created_ns"] for i in tn])]
        assert r["order"][(g, 0)] == oldest
        assert r["order"][(g, 1)] == newest
        # RunOnce's selections (slack 1): the walk's first nodes, delivered with the decision
        which, sel = r["select"][g]
        if L["delta"] > 0:
            assert which == 1 and sel == newest[:L["delta"] + 1], (g, which, sel)
        elif L["delta"] < 0 and not L["taint_err"]:
            assert which == 0 and sel == oldest[:L["n_to_taint"] + 1], (g, which, sel)
        else:
            assert which == -1 and sel == [], (g, which, sel)
    try:
        mem, cpu = O.calculate_pods_requests_total(pods)
        assert r["list_pods"] == (mem, cpu)
    except O.QuantityOverflow:
        assert r["list_pods"] is None
    assert r["list_nodes"] == O.calculate_nodes_capacity_total(nodes)
