"""CPU: K0 packer (product, host C++) -> packed SoA -> C oracle, against the literal
Python oracle on the original objects.  Pins the C oracle (used at full sizes) to the
fixture-pinned literal oracle, and checks the packer's encoding without a GPU."""
import random
import struct

import numpy as np
import pytest

from oracle import oracle as O
from oracle import soa
from randobj import make_groups, make_nodes, make_pods, make_reaping_cluster, make_states, make_trackers

soa.build()


def _ctx(groups):
    from escalator_amd.context import Context
    return Context(groups, device=-1)


def literal_all(groups, states, pods, nodes, trackers):
    out = []
    for g, spec in enumerate(groups):
        out.append(O.scale_node_group(spec, states[g], pods, nodes, tracker=trackers.get(g, [])))
    return out


def _bits(x):
    return struct.pack("<d", x)


def compare(groups, states, pods, nodes, trackers, tot, df, di):
    lit = literal_all(groups, states, pods, nodes, trackers)
    for g, L in enumerate(lit):
        t = tot[g]
        assert t[2] == L["n_pods"], (g, "n_pods")
        assert (t[5], t[6], t[7], t[8]) == (L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"]), g
        assert t[9] == L["first_node"], g
        if L["pod_cpu_m"] is not None:
            assert (t[0], t[1], t[3], t[4]) == (L["pod_cpu_m"], L["pod_mem_b"], L["node_cpu_m"], L["node_mem_b"]), g
            assert t[12] == 0
        else:
            assert t[12] != 0
        assert soa.BRANCH_NAMES[di[g, 5]] == L["branch"], (g, L)
        assert soa.STATUS_ERR[di[g, 4]] == L["err"], (g, L)
        assert di[g, 0] == L["delta"], (g, L)
        assert _bits(df[g, 0]) == _bits(L["cpu_pct"]) and _bits(df[g, 1]) == _bits(L["mem_pct"]), (g, L)
        assert (di[g, 2], di[g, 3]) == (L["cached_cpu_m"], L["cached_mem_b"]), g
        assert di[g, 1] == L["n_to_taint"] and (di[g, 6] != 0) == (L["taint_err"] is not None), (g, L)


@pytest.mark.parametrize("seed", range(16))
def test_packer_c_oracle_vs_literal(seed):
    rng = random.Random(1000 + seed)
    G = rng.choice([1, 3, 8, 20])
    groups = make_groups(rng, G, with_default=rng.random() < 0.6)
    pods = make_pods(rng, rng.choice([0, 60, 400]) if seed else 0, groups)
    nodes = make_nodes(rng, rng.choice([10, 40, 120]) if seed else 0, groups)
    trackers = make_trackers(rng, groups, nodes)
    states = make_states(rng, G)
    ctx = _ctx(groups)
    P, N = ctx.pack(pods, nodes, trackers)
    tot = soa.totals(P, N, groups)
    df, di = soa.decide(groups, states, tot)
    compare(groups, states, pods, nodes, trackers, tot, df, di)
    # reference-shaped scan gives identical totals
    assert np.array_equal(soa.totals(P, N, groups, reference_shaped=True), tot)
    # orderings
    for g in range(G):
        L = O.scale_node_group(groups[g], states[g], pods, nodes, tracker=trackers.get(g, []))
        unt = L["untainted"]
        want = [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
        assert list(soa.order(N, groups, g, 0)) == want
        tn = L["tainted"]
        want = [tn[i] for i in O.newest_first([nodes[i]["created_ns"] for i in tn])]
        assert list(soa.order(N, groups, g, 1)) == want


@pytest.mark.parametrize("seed", range(8))
def test_c_oracle_try_remove_vs_literal(seed):
    """orc_try_remove (used at full sizes) equals the fixture-pinned literal
    TryRemoveTaintedNodes on random clusters, through the packer's pod / node order."""
    from escalator_amd.objects import placement
    rng = random.Random(4400 + seed)
    G = rng.choice([1, 4, 12])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, rng.choice([0, 200, 800]), rng.choice([5, 50, 150]))
    trackers = make_trackers(rng, groups, nodes)
    P, N = _ctx(groups).pack(pods, nodes, trackers)
    pn, ts, nd = placement(pods, nodes)
    for g, grp in enumerate(groups):
        soft, hard = rng.choice([0, 60, 300]) * 10**9, rng.choice([300, 900]) * 10**9
        L = O.scale_node_group(grp, {}, pods, nodes, tracker=trackers.get(g, []))
        pods_g = O.filtered_list(pods, O.group_pod_filter(grp))
        all_nodes = [n for n in nodes
                     if O.new_node_label_filter_func(grp.get("label_key", ""), grp.get("label_value", ""))(n)]
        tainted = L["tainted"]
        neg, rem, ks = O.try_remove_tainted_nodes(grp, [nodes[i] for i in tainted], pods_g, all_nodes, now_ns,
                                                  soft, hard, bool(grp.get("dry_mode")))
        res, idx = soa.try_remove(P, N, groups, pn, ts, nd, g, now_ns, soft, hard)
        assert res == (len(tainted), -neg, rem), g
        assert list(idx) == [tainted[k] for k in ks], g


def test_packer_list_mode_fixtures(golden):
    from builders import build_test_node, build_test_pod
    fx = golden["k8s_util"]
    ctx = _ctx([{"name": "x", "label_key": "k", "label_value": "v"}])
    for c in fx["calculate_pods_requests_total"]:
        pods = [build_test_pod(fx["pods"][n]) for n in c["pods"]]
        P, N = ctx.pack(pods, [], list_mode=True)
        tot = soa.totals(P, N, [{"name": "x"}])
        assert (tot[0, 1], tot[0, 0]) == (c["mem"], c["cpu"]), c["name"]
    for c in fx["calculate_nodes_capacity_total"]:
        nodes = [build_test_node(fx["nodes"][n]) for n in c["nodes"]]
        P, N = ctx.pack([], nodes, list_mode=True)
        tot = soa.totals(P, N, [{"name": "x"}])
        assert (tot[0, 4], tot[0, 3]) == (c["mem"], c["cpu"]), c["name"]


def test_packer_encoding_details():
    groups = [{"name": "default", "label_key": "customer", "label_value": "default"},
              {"name": "a", "label_key": "customer", "label_value": "a"},
              {"name": "b", "label_key": "customer", "label_value": "a"},
              {"name": "c", "label_key": "pool", "label_value": "p"}]
    ctx = _ctx(groups)
    pods = [
        {"containers": [{"cpu": 5, "mem": 6}], "node_selector": {"customer": "a", "pool": "p"},
         "affinity": {"node_affinity": {"required": [[{"key": "customer", "op": "In", "values": ["a", "zz"]}]]}}},
        {"containers": [{"cpu": 1 << 33, "mem": 1}, {"cpu": 2, "mem": 3}], "init_containers": [{"cpu": None, "mem": 9}],
         "overhead": {"cpu": None, "mem": None}},
        {"owner_kinds": ["DaemonSet"], "containers": []},
    ]
    P, N = ctx.pack(pods, [])
    # pair ids (numbering rule): (customer,default)=0, (customer,a)=1 shared by groups a and b,
    # (pool,p)=2; (customer,zz) is a group-key value no group has -> first packer id, 3.
    # pod 0 carries {1, 2, 3}, deduped across selector + affinity; group resolution is K1's
    assert P["pair0"][0] == 1 and list(P["xp_pair"]) == [2, 3]
    assert (P["flags"][0] >> 24) & 63 == 2 and P["flags"][0] & 0b1100 == 0b1100
    # pod 1: first container cpu does not fit u32 -> all regulars are extras; absent init cpu = INT64_MIN;
    # an overhead map with no keys adds nothing and is dropped
    assert P["cpu0"][1] == 0 and (P["flags"][1] >> 8) & 255 == 2 and (P["flags"][1] >> 16) & 255 == 1
    assert not P["flags"][1] & 16
    assert list(P["xc_cpu"]) == [1 << 33, 2, -(1 << 63)] and list(P["xc_mem"]) == [1, 3, 9]
    assert P["pair0"][1] == 0xFFFFFFFF
    assert P["flags"][2] & 1


def test_scalar_math_matches_literal():
    """The library's host build of the decision math (same code as the K4 kernel)."""
    import ctypes as C
    from escalator_amd import _lib as L
    lib = L.load()
    rng = random.Random(5)
    cases = [(50, 50, 100, 100, 1), (50, 50, 0, 0, 10), (0, 0, 0, 0, 1), (0, 0, 66, 66, 1), (0, 0, 0, 0, 0),
             (50000, 60000, 15000, 50000, 10)]
    for _ in range(3000):
        cases.append((rng.randrange(-10, 1 << 62), rng.randrange(0, 1 << 62), rng.choice([0, rng.randrange(1, 1 << 62)]),
                      rng.choice([0, rng.randrange(1, 1 << 60)]), rng.randrange(0, 3)))
    a, b = C.c_double(), C.c_double()
    for c in cases:
        st = lib.esc_calc_percent_usage(*c, C.byref(a), C.byref(b))
        cpu, mem, err = O.calc_percent_usage(*c)
        assert _bits(a.value) == _bits(cpu) and _bits(b.value) == _bits(mem), c
        assert (st == 3) == (err is not None)
        d = C.c_int64()
        for thr in (0, 1, 3, 70, 110):
            for cached in ((0, 0), (4000, 8 << 30)):
                st = lib.esc_calc_scale_up_delta(c[4], a.value, b.value, c[0], c[1], cached[0], cached[1], thr,
                                                 C.byref(d))
                want, err = O.calc_scale_up_delta(c[4], a.value, b.value, c[0], c[1], cached[0], cached[1], thr)
                assert d.value == want and (st == 4) == (err is not None), (c, thr, cached)


def test_packer_over_generator_objects_equals_generator():
    """The generator's snapshot as object structs (esc_synth_objects: owner kinds, the
    config.source annotation, nodeSelector, required node-affinity "In" / "NotIn"
    expressions, PodAffinity, containers, labels, cordon, taints, allocatable) packed by K0
    gives the generator's packed snapshot's totals for every group (the pair ids of values
    no group selects are numbered differently, which no filter can see)."""
    from escalator_amd.context import Context, Synth
    for cfg, P, N, G in ((2, 60_000, 2_000, 100), (4, 40_000, 3_000, 700), (3, 30_000, 1_000, 20)):
        s = Synth(P, N, G, config=cfg, seed=cfg + 40, threads=4)
        po, n, no, nn = s.objects()
        assert (n, nn) == (P, N)
        nodes = s.nodes()
        trk = {}
        for j, g in zip(nodes["trk_node"], nodes["trk_group"]):
            trk.setdefault(int(g), []).append("node-%d" % j)
        ctx = Context(s.groups, device=-1)
        Pk, Nk = ctx.pack_objects(po, n, no, nn, trk)
        pods = s.pods()
        assert np.array_equal(Pk["pair0"] < 0x7FFFFFFF, pods["pair0"] < 0x7FFFFFFF)
        assert np.array_equal(soa.totals(Pk, Nk, s.groups), soa.totals(pods, nodes, s.groups)), cfg


_PACKER_CHILD = r"""
import json, os, random, sys
sys.path[:0] = [sys.argv[1], os.path.join(sys.argv[1], "tests")]
from randobj import make_groups, make_nodes, make_pods, make_trackers
from escalator_amd.context import Context
rng = random.Random(int(sys.argv[2]))
groups = make_groups(rng, 12, with_default=True)
pods = make_pods(rng, 3000, groups)
nodes = make_nodes(rng, 900, groups)
trackers = make_trackers(rng, groups, nodes)
P, N = Context(groups, device=-1).pack(pods, nodes, trackers)
print(json.dumps({k: v.tolist() for k, v in list(P.items()) + [("n_" + k, v) for k, v in N.items()]}))
"""


@pytest.mark.parametrize("seed", range(3))
def test_parallel_packer_equals_sequential(seed):
    """The packer's multi-threaded path (parts packed per thread, provisional ids for values
    no group selects, renumbered in chunk order at the merge) gives the sequential packer's
    arrays exactly — pair ids included — on objects full of such values."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(threads, par_min):
        env = dict(os.environ, ESC_HOST_THREADS=str(threads), ESC_PACK_PAR_MIN=str(par_min))
        r = subprocess.run([sys.executable, "-c", _PACKER_CHILD, root, str(seed)], env=env,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        return json.loads(r.stdout)

    seq = run(1, 1 << 30)
    for threads in (2, 7):
        par = run(threads, 16)
        assert par.keys() == seq.keys()
        for k in seq:
            assert par[k] == seq[k], (threads, k)
    assert any(q >= 12 for q in seq["xp_pair"] + seq["pair0"] if q != 0xFFFFFFFF)   # values no group selects
