"""GPU parity tests: the HIP path (through the C ABI) against the oracles.

Bit-exact everywhere: int64 sums and counts, float64 percentages compared as bits,
deltas, statuses and node orderings."""
import ctypes as C
import random
import struct

import numpy as np
import pytest

from builders import build_test_node, build_test_nodes, build_test_pod, build_test_pods, unix_ns
from oracle import oracle as O
from oracle import soa
from randobj import make_groups, make_nodes, make_pods, make_reaping_cluster, make_states, make_trackers

pytestmark = pytest.mark.gpu
soa.build()


def _bits(x):
    return struct.pack("<d", float(x))


@pytest.fixture(scope="module")
def esc():
    import escalator_amd
    return escalator_amd


def check_metrics(m, expected):
    """GPU gauges (esc_metrics_results) == the oracle's, bit for bit, and the same set mask."""
    from escalator_amd._lib import METRIC_NAMES
    for g, e in enumerate(expected):
        mask = sum(1 << k for k, n in enumerate(METRIC_NAMES) if n in e)
        assert int(m["set_mask"][g]) == mask, (g, e)
        for n, v in e.items():
            assert _bits(m[n][g]) == _bits(v), (g, n, m[n][g], v)


def check_against_c_oracle(tot, dec, otot, odf, odi):
    names = list(tot.dtype.names)
    for k, name in enumerate(soa.TOT_FIELDS):
        if name == "flags":
            assert np.array_equal(tot[name] != 0, otot[:, k] != 0), name
            continue
        assert np.array_equal(tot[name], otot[:, k]), (name, np.nonzero(tot[name] != otot[:, k])[0][:10])
    assert names
    assert np.array_equal(dec["cpu_pct"].view(np.uint64), odf[:, 0].view(np.uint64))
    assert np.array_equal(dec["mem_pct"].view(np.uint64), odf[:, 1].view(np.uint64))
    for k, name in enumerate(["delta", "n_to_taint", "cached_cpu_m", "cached_mem_b", "status", "branch",
                              "taint_status"]):
        assert np.array_equal(dec[name].astype(np.int64), odi[:, k]), (name, np.nonzero(dec[name] != odi[:, k])[0][:10])


# ------------------------------------------------------------------ fixtures
def test_fixture_pods_requests_total(esc, golden):
    from escalator_amd import k8s
    fx = golden["k8s_util"]
    for c in fx["calculate_pods_requests_total"]:
        pods = [build_test_pod(fx["pods"][n]) for n in c["pods"]]
        assert k8s.calculate_pods_requests_total(pods) == (c["mem"], c["cpu"]), c["name"]


def test_fixture_nodes_capacity_total(esc, golden):
    from escalator_amd import k8s
    fx = golden["k8s_util"]
    for c in fx["calculate_nodes_capacity_total"]:
        nodes = [build_test_node(fx["nodes"][n]) for n in c["nodes"]]
        assert k8s.calculate_nodes_capacity_total(nodes) == (c["mem"], c["cpu"]), c["name"]


@pytest.mark.parametrize("seed", range(3))
def test_dropin_lists_vs_literal(esc, seed):
    """The per-call drop-ins (esc_list.hip: pinned buffers reused across calls, one kernel)
    over random slices — absent / zero / negative / huge requests, init containers,
    overhead, daemonsets (the Go functions take the slice as given: no filter) — equal the
    literal CalculatePodsRequestsTotal / CalculateNodesCapacityTotal; sizes from empty to
    many workgroups, repeated calls on one context, growth of the buffers; a total outside
    int64 raises OverflowError (the reference's Quantity would move to inf.Dec)."""
    from escalator_amd import k8s
    rng = random.Random(8800 + seed)
    groups = make_groups(rng, 3, with_default=True)
    for n in (0, 1, 7, 1000, 3000, 40_000, 1000):
        pods = make_pods(rng, n, groups, big_frac=0.05 if n < 5000 else 0.0)
        try:
            want = O.calculate_pods_requests_total(pods)
        except O.QuantityOverflow:
            want = None
        if want is None:
            t = [O.compute_pod_resource_request(p) for p in pods]
            exact = (sum(m for _, m in t), sum(c for c, _ in t))
            if all(-(1 << 63) <= v < (1 << 63) for v in exact):
                want = exact                    # order-independent exact total (unpinned: see DESIGN.md §2)
        if want is None:
            with pytest.raises(OverflowError):
                k8s.calculate_pods_requests_total(pods)
        else:
            assert k8s.calculate_pods_requests_total(pods) == want, n
        nodes = make_nodes(rng, max(n // 20, 0), groups, big_frac=0.0)
        assert k8s.calculate_nodes_capacity_total(nodes) == O.calculate_nodes_capacity_total(nodes), n
    big = [build_test_pod({"CPU": [1 << 62], "Mem": [1 << 62]})] * 3
    with pytest.raises(OverflowError):
        k8s.calculate_pods_requests_total(big)


def test_fixture_orderings(esc, golden):
    from escalator_amd import controller
    fx = golden["controller"]
    dates = [unix_ns(*d) for d in fx["six_nodes"]["dates"]]
    for c in fx["taint_oldest_n"]:
        assert controller.taint_oldest_n(dates[:c["slice"]], c["n"]) == c["want"], c["name"]
    for c in fx["untaint_newest_n"]:
        assert controller.untaint_newest_n(dates[:c["slice"]], c["n"]) == c["want"], c["name"]
    old = [unix_ns(*d) for d in fx["sort_dates"]["oldest_ordered"]]
    rng = random.Random(3)
    for _ in range(10):
        perm = list(range(6))
        rng.shuffle(perm)
        got = controller.taint_oldest_n([old[i] for i in perm], 6)
        assert [perm[i] for i in got] == list(range(6))


def _default_group(opts):
    g = {"name": "default", "label_key": "", "label_value": ""}
    g.update(opts)
    g.setdefault("max_nodes", 0)
    return g


def test_fixture_scale_node_group(esc, golden):
    from escalator_amd.controller import Controller
    for c in golden["controller"]["scale_node_group"]["cases"]:
        n_n, n_cpu, n_mem = c["nodes"]
        n_p, p_cpu, p_mem = c["pods"]
        nodes = build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem})
        pods = build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]})
        ctl = Controller([_default_group(c["opts"])])

        def lp():
            if c.get("lister_error") == "pods":
                raise RuntimeError("unable to list pods")
            return pods

        def ln():
            if c.get("lister_error") == "nodes":
                raise RuntimeError("unable to list nodes")
            return nodes

        delta, err = ctl.scale_node_group("default", lp, ln)
        assert (delta, err) == (c["delta"], c["err"]), c["name"]
        if delta > 0:                       # re-run after the cloud brought the nodes up -> 0
            more = nodes + build_test_nodes(delta, {"CPU": n_cpu, "Mem": n_mem}, "m")
            assert ctl.scale_node_group("default", lambda: pods, lambda: more)[0] == 0, c["name"]


def test_fixture_multiple_runs_first_delta(esc, golden):
    from escalator_amd.controller import Controller
    for c in golden["controller"]["scale_node_group_multiple_runs"]["cases"]:
        n_n, n_cpu, n_mem = c["nodes"]
        n_p, p_cpu, p_mem = c["pods"]
        nodes = build_test_nodes(n_n, {"CPU": n_cpu, "Mem": n_mem})
        pods = build_test_pods(n_p, {"CPU": [p_cpu], "Mem": [p_mem]})
        ctl = Controller([_default_group(c["opts"])])
        if c["cached"]:
            ctl.state[0]["cached_cpu_m"], ctl.state[0]["cached_mem_b"] = c["cached"]
        assert ctl.scale_node_group("default", lambda: pods, lambda: nodes) == (c["delta"], None), c["name"]


def test_fixture_filter_nodes_dry_and_wet(esc, golden):
    fx = golden["controller"]["filter_nodes"]
    nodes = [build_test_node(o) for o in fx["nodes"]]
    for c in fx["cases"]:
        g = {"name": "g", "label_key": "", "label_value": "", "max_nodes": 100, "dry_mode": c["dry"]}
        ctx = esc.Context([g])
        P, N = ctx.pack([], nodes, {0: c["tracker"]} if c["tracker"] else None)
        ctx.load(P, N)
        tot, _ = ctx.decide_all()
        assert (tot["n_untainted"][0], tot["n_tainted"][0], tot["n_cordoned"][0]) == \
            (len(c["untainted"]), len(c["tainted"]), len(c["cordoned"]))
        ctx.sort_nodes()
        assert list(ctx.group_order(0, 0)) == c["untainted"]
        assert sorted(ctx.group_order(0, 1)) == c["tainted"]


# ------------------------------------------------------ random object clusters
@pytest.mark.parametrize("seed", range(10))
def test_random_objects_vs_literal(esc, seed):
    rng = random.Random(2000 + seed)
    G = rng.choice([1, 3, 8, 20])
    groups = make_groups(rng, G, with_default=rng.random() < 0.6)
    pods = make_pods(rng, rng.choice([0, 60, 500]) if seed else 0, groups, big_frac=0.03)
    nodes = make_nodes(rng, rng.choice([10, 40, 150]) if seed else 0, groups, big_frac=0.03)
    trackers = make_trackers(rng, groups, nodes)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    ctx.set_metrics(True)
    for wide in (False, True):
        ctx.force_wide(wide)
        tot, dec = ctx.decide_all(states)
        check_metrics(ctx.metrics(), [O.node_group_metrics(O.scale_node_group(groups[g], states[g], pods, nodes,
                                                                              tracker=trackers.get(g, [])))
                                      for g in range(G)])
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], pods, nodes, tracker=trackers.get(g, []))
            t, d = tot[g], dec[g]
            assert (t["n_pods"], t["n_nodes"], t["n_untainted"], t["n_tainted"], t["n_cordoned"], t["first_node"]) == \
                (L["n_pods"], L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"], L["first_node"]), g
            if L["pod_cpu_m"] is not None:
                assert (t["pod_cpu_m"], t["pod_mem_b"], t["node_cpu_m"], t["node_mem_b"]) == \
                    (L["pod_cpu_m"], L["pod_mem_b"], L["node_cpu_m"], L["node_mem_b"]), g
            assert esc._lib.BRANCHES[d["branch"]] == L["branch"], (g, L)
            assert int(d["delta"]) == L["delta"] and int(d["n_to_taint"]) == L["n_to_taint"], (g, L)
            assert _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]) and _bits(d["mem_pct"]) == _bits(L["mem_pct"])
            assert (int(d["cached_cpu_m"]), int(d["cached_mem_b"])) == (L["cached_cpu_m"], L["cached_mem_b"])
    ctx.force_wide(False)
    ctx.sort_nodes()
    for g in range(G):
        L = O.scale_node_group(groups[g], states[g], pods, nodes, tracker=trackers.get(g, []))
        unt = L["untainted"]
        assert list(ctx.group_order(g, 0)) == [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
        tn = L["tainted"]
        assert list(ctx.group_order(g, 1)) == [tn[i] for i in O.newest_first([nodes[i]["created_ns"] for i in tn])]


def test_overflow_flagged(esc):
    groups = [{"name": "a", "label_key": "k", "label_value": "v", "max_nodes": 10}]
    pods = [{"containers": [{"cpu": 1, "mem": (1 << 62) + 5}], "node_selector": {"k": "v"}} for _ in range(3)]
    nodes = [{"name": "n", "labels": {"k": "v"}, "cpu": 1000, "mem": 1000, "created_ns": 1}]
    ctx = esc.Context(groups)
    ctx.load(*ctx.pack(pods, nodes))
    tot, dec = ctx.decide_all()
    assert tot["flags"][0] & 1 and dec["status"][0] == esc._lib.ESC_ST_ERR_OVERFLOW


# ---------------------------------------------------------- synthetic configs
@pytest.mark.parametrize("cfg,P,N,G", [(1, 1000, 50, 1), (2, 1_000_000, 10_000, 100), (3, 2_000_000, 20_000, 100),
                                       (4, 2_000_000, 20_000, 10_000), (5, 200_000, 300_000, 100)])
def test_synthetic_vs_c_oracle(esc, cfg, P, N, G):
    s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg)
    pods, nodes = s.pods(), s.nodes()
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(True)
    ctx.set_state(s.states)
    for _ in range(3):                        # graph replays over both replicas
        ctx.run()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    assert len(set(dec["branch"].tolist())) >= (1 if G == 1 else 3)
    ctx.force_wide(True)
    ctx.run()
    tot, dec = ctx.results()
    check_against_c_oracle(tot, dec, otot, odf, odi)
    ctx.force_wide(False)
    ctx.set_metrics(True)
    ctx.run()
    check_metrics(ctx.metrics(), soa.metrics(otot, odf, odi))


@pytest.mark.parametrize("cfg,P,N,G", [(2, 1_000_000, 10_000, 100), (4, 2_000_000, 20_000, 10_000),
                                       (4, 300, 50, 10_000), (1, 1000, 50, 1)])
def test_step_graph_and_wide_vs_c_oracle(esc, cfg, P, N, G):
    """The step (K1, the fused tail k_step_tail: fold + node pieces, then node groups +
    decide) gives bit-exact totals and decisions over repeated graph replays and with the
    exact wide path forced in between (the wide rows are read and reset by the fold)."""
    s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg)
    otot = soa.totals(s.pods(), s.nodes(), s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(True)
    ctx.set_state(s.states)
    for k in range(5):
        ctx.force_wide(k == 2)
        ctx.run()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)


@pytest.mark.parametrize("cfg,P,N,G", [(4, 2_000_000, 20_000, 10_000), (2, 1_000_000, 10_000, 100),
                                       (3, 2_000_000, 20_000, 100)])
def test_k1_calibrated_shares_vs_c_oracle(esc, cfg, P, N, G):
    """esc_k1_calibrate moves K1's per-workgroup shares to the measured rates: the plan
    changes, every tile is still taken exactly once (totals and decisions bit-exact before
    and after, through the captured graph, which reads the plan from device memory), and
    the per-workgroup K phase is timed (trace words 0-1)."""
    s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg)
    otot = soa.totals(s.pods(), s.nodes(), s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(True)
    ctx.set_state(s.states)
    ctx.run()
    check_against_c_oracle(*ctx.results(), otot, odf, odi)
    ctx.k1_calibrate(3)
    tr = ctx.k1_trace()
    assert tr.shape[0] > 1 and np.all(tr[:, 1] >= tr[:, 0])
    for _ in range(3):
        ctx.run()
        check_against_c_oracle(*ctx.results(), otot, odf, odi)


def test_synthetic_sort_vs_c_oracle(esc):
    """The K5 per-decision ordering (two passes over the groups' split chunks, several
    chunks per group here), repeated decisions and a dry-mode tracker change in between."""
    s = esc.Synth(10_000, 400_000, 100, config=5, seed=0xE5CA1A7E00000005)
    nodes = s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s)
    for _ in range(3):
        ctx.sort_nodes()
    for g in list(range(0, 100, 7)) + [99]:
        for which in (0, 1):
            assert np.array_equal(ctx.group_order(g, which), soa.order(nodes, s.groups, g, which)), (g, which)
    # a dry group's tracker changes in place; its split follows the new tracker
    g = next(g for g, x in enumerate(s.groups) if x.get("dry_mode"))
    members = _members_oldest(nodes, s.groups, g)
    ctx.tracker_update(g, add=ctx.group_order(g, 0)[:500], remove=ctx.group_order(g, 1)[:100])
    ctx.sort_nodes()
    trk = set(ctx.tracker_list(g).tolist())
    t = nodes["created_ns"]
    assert ctx.group_order(g, 0).tolist() == [j for j in members if j not in trk]
    assert ctx.group_order(g, 1).tolist() == sorted((j for j in members if j in trk), key=lambda j: (-int(t[j]), j))


@pytest.mark.parametrize("N", [1, 15, 17, 2_047, 2_049, 8_191, 8_193, 40_000, 1_100_000])
def test_age_index_sizes_vs_c_oracle(esc, N):
    """The age index's LSD scatter at memberships around its line (16 keys), chunk (2048)
    and block (8192) sizes and at several chunks per block: each chunk writes whole lines of
    a digit's run and carries the partial last line to the next (esc_kernels.hip
    k_rs_scatter, ESC_RS_CARRY); every group's orderings against the C oracle."""
    s = esc.Synth(max(1, N // 4), N, 7, config=5, seed=0xE5CA1A7E00000100 + N)
    nodes = s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.sort_nodes()
    for g in range(len(s.groups)):
        for which in (0, 1):
            assert np.array_equal(ctx.group_order(g, which), soa.order(nodes, s.groups, g, which)), (N, g, which)


@pytest.mark.parametrize("run", [2, 8, 9, 64])
def test_age_index_coarse_key_runs_vs_c_oracle(esc, run):
    """The age index's 32-bit coarse keys: with the creation range widened
    past the bits a key keeps, `run` members of one group share ONE timestamp and `run` more
    lie within one coarse-key bucket (times descending with the index).  Runs of <= 8 equal
    coarse keys are ordered exactly by k_age_fix; a longer run sends the build back to the
    exact 64-bit keys.  Every group's two orders against the C oracle, before and after a
    rebuild."""
    s = esc.Synth(2_000, 20_000, 7, config=5, seed=0xE5CA1A7E00000200 + run)
    pods = s.pods()
    nodes = {k: np.array(v, copy=True) for k, v in s.nodes().items()}
    t = nodes["created_ns"]
    t[0] = int(t.min()) - (1 << 37) - 1              # range > 2^37 ns, divisor 1: bits dropped
    m = [j for j in _members_oldest(nodes, s.groups, 1) if j != 0]
    assert len(m) >= 2 * run
    mid = int(np.median(t))
    t[m[:run]] = mid + 7                              # exact ties: equal keys at any width
    t[m[run:2 * run]] = mid + (1 << 30) + np.arange(run)[::-1]   # one bucket, times falling
    ctx = esc.Context(s)
    ctx.load(pods, nodes)
    for _ in range(2):
        ctx.sort_nodes()
        for g in range(len(s.groups)):
            for which in (0, 1):
                assert np.array_equal(ctx.group_order(g, which), soa.order(nodes, s.groups, g, which)), (run, g, which)
        ctx.build_age_index()


@pytest.mark.parametrize("graph,N", [(False, 200_000), (True, 200_000), (True, 30_000), (True, 700_000)])
def test_order_in_step_vs_c_oracle(esc, graph, N):
    """esc_set_order_in_step: the K5 ordering inside every decision (side stream beside K1,
    captured in the decision graph) — orders valid after esc_run with no esc_sort_nodes,
    also after node events patch the flags, and the decision itself unchanged.  Group sizes
    cover the packed chunk kinds (<= 1024 and <= 4096 memberships) and the split one."""
    s = esc.Synth(300_000, N, 100, config=5, seed=0xE5CA1A7E00000005)
    pods, nodes = s.pods(), s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(graph)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    for _ in range(3):
        ctx.run()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    full = soa.order_all(nodes, s.groups)
    for g in range(100):
        for which in (0, 1):
            assert np.array_equal(ctx.group_order(g, which), full[(g, which)]), (g, which)
    # node events (cordon / taint flips) then one more decision: orders follow the flags
    rng = np.random.default_rng(5)
    ids = rng.choice(len(nodes["flags"]), min(2000, N // 10), replace=False).astype(np.int64)
    flags = nodes["flags"].copy()
    flags[ids] ^= rng.integers(1, 4, len(ids)).astype(np.uint32) & 3
    ctx.nodes_update(ids, flags[ids], nodes["cpu"][ids], nodes["mem"][ids])
    n2 = dict(nodes, flags=flags)
    ctx.run()
    ctx.results()
    full = soa.order_all(n2, s.groups)
    for g in range(0, 100, 3):
        for which in (0, 1):
            assert np.array_equal(ctx.group_order(g, which), full[(g, which)]), (g, which)
    # an explicit index rebuild, then decisions through the (re)captured step: the ordering's
    # status arrays alternate by decision parity, so run an odd and an even number
    ctx.build_age_index()
    for k in range(3):
        ctx.run()
        ctx.results()
        for g in range(k, 100, 7):
            for which in (0, 1):
                assert np.array_equal(ctx.group_order(g, which), full[(g, which)]), (k, g, which)


@pytest.mark.parametrize("seed", range(6))
def test_node_add_delete_vs_literal(esc, seed):
    """Node informer Add / Delete events in place (esc_nodes_add / esc_nodes_delete): after
    every round of deletions and additions (creation times older, newer and equal to the
    loaded ones), the totals, allNodes[0], decisions and both orderings equal the literal
    oracle over the live nodes in snapshot order; half the seeds decide through the graph
    with the ordering in the step."""
    rng = random.Random(9100 + seed)
    G = rng.choice([3, 8, 20])
    groups = make_groups(rng, G, with_default=rng.random() < 0.6)
    pods = make_pods(rng, 300, groups, big_frac=0.0)
    nodes = make_nodes(rng, rng.choice([40, 120]), groups, big_frac=0.0)
    trackers = make_trackers(rng, groups, nodes)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    ctx.set_spare(1.0)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    in_step = seed % 2 == 1
    if in_step:
        ctx.use_graph(True)
        ctx.set_order_in_step(True)
    live = dict(enumerate(nodes))
    pflags = {j: int(N["flags"][j]) for j in live}
    hw = base = len(nodes)
    for rnd in range(5):
        dels = rng.sample(sorted(live), k=min(len(live), rng.randrange(0, 12)))
        if dels:
            ctx.nodes_delete(dels)
            for j in dels:
                del live[j]
        new = make_nodes(rng, rng.randrange(0, 14), groups, big_frac=0.0)
        for k, nd in enumerate(new):
            nd["name"] = "r%d-new%d" % (rnd, k)
        if new:
            _, packed = ctx.pack([], new)
            try:
                ids = ctx.nodes_add(packed)
            except esc._lib.EscError as e:                            # spare room short: reload
                assert e.code == esc._lib.ESC_E_LIMIT
                lst = [live[j] for j in sorted(live)] + new
                P, N = ctx.pack(pods, lst, trackers)
                ctx.load(P, N)
                live = dict(enumerate(lst))
                pflags = {j: int(N["flags"][j]) for j in live}
                hw = base = len(lst)
            else:
                assert list(ids) == list(range(hw, hw + len(new)))      # next snapshot indices
                hw += len(new)
                for k, (j, nd) in enumerate(zip(ids, new)):
                    live[int(j)] = nd
                    pflags[int(j)] = int(packed["flags"][k])
        idx = sorted(live)
        lst = [live[j] for j in idx]
        tot, dec = ctx.decide_all(states)
        if not in_step:
            ctx.sort_nodes()
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], pods, lst, tracker=trackers.get(g, []))
            t, d = tot[g], dec[g]
            first = idx[L["first_node"]] if L["first_node"] >= 0 else -1
            assert (t["n_pods"], t["n_nodes"], t["n_untainted"], t["n_tainted"], t["n_cordoned"], t["first_node"]) == \
                (L["n_pods"], L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"], first), (rnd, g)
            if L["pod_cpu_m"] is not None:
                assert (t["node_cpu_m"], t["node_mem_b"]) == (L["node_cpu_m"], L["node_mem_b"]), (rnd, g)
            assert esc._lib.BRANCHES[d["branch"]] == L["branch"], (rnd, g)
            assert int(d["delta"]) == L["delta"] and int(d["n_to_taint"]) == L["n_to_taint"], (rnd, g)
            assert _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]) and _bits(d["mem_pct"]) == _bits(L["mem_pct"])
            assert (int(d["cached_cpu_m"]), int(d["cached_mem_b"])) == (L["cached_cpu_m"], L["cached_mem_b"])
            unt, tn = L["untainted"], L["tainted"]
            assert list(ctx.group_order(g, 0)) == \
                [idx[unt[i]] for i in O.oldest_first([lst[k]["created_ns"] for k in unt])], (rnd, g)
            assert list(ctx.group_order(g, 1)) == \
                [idx[tn[i]] for i in O.newest_first([lst[k]["created_ns"] for k in tn])], (rnd, g)
    # cordon / taint updates of added nodes, then a full rebuild of the age index agrees
    added = [j for j in live if j >= base]
    if added:
        flags = np.array([pflags[j] | 2 for j in added], np.uint32)      # + the escalator taint
        cpu = np.array([live[j].get("cpu") or 0 for j in added], np.int64)
        mem = np.array([live[j].get("mem") or 0 for j in added], np.int64)
        ctx.nodes_update(np.array(added, np.int64), flags, cpu, mem)
        for j in added:
            live[j] = dict(live[j], taints=["atlassian.com/escalator"])
        ctx.decide_all(states)
        if not in_step:
            ctx.sort_nodes()
        before = {(g, w): list(ctx.group_order(g, w)) for g in range(G) for w in (0, 1)}
        ctx.build_age_index()
        ctx.sort_nodes()
        assert before == {(g, w): list(ctx.group_order(g, w)) for g in range(G) for w in (0, 1)}


def _relabel(rng, nd, groups, move_time):
    """A node Update with new labels (group moves, extra labels, labels no group uses), maybe
    a new creation time, taint / cordon and allocatable."""
    x = make_nodes(rng, 1, groups, big_frac=0.0)[0]
    x["name"] = nd["name"]
    for k in ("taint_value", "annotations"):
        if k in nd:
            x[k] = nd[k]
    if not move_time:
        x["created_ns"] = nd["created_ns"]
    elif rng.random() < 0.3:
        x["created_ns"] = nd["created_ns"] + rng.choice([-1, 1]) * rng.randrange(1, 5) * 1_000
    return x


def _check_nodes_vs_literal(ctx, groups, states, pods, live, trackers, tag):
    idx = sorted(live)
    lst = [live[j] for j in idx]
    tot, dec = ctx.decide_all(states)
    ctx.sort_nodes()
    for g in range(len(groups)):
        L = O.scale_node_group(groups[g], states[g], pods, lst, tracker=trackers.get(g, []))
        t, d = tot[g], dec[g]
        first = idx[L["first_node"]] if L["first_node"] >= 0 else -1
        assert (t["n_pods"], t["n_nodes"], t["n_untainted"], t["n_tainted"], t["n_cordoned"], t["first_node"]) == \
            (L["n_pods"], L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"], first), (tag, g)
        if L["pod_cpu_m"] is not None:
            assert (t["node_cpu_m"], t["node_mem_b"]) == (L["node_cpu_m"], L["node_mem_b"]), (tag, g)
        assert esc_branch(d) == L["branch"], (tag, g)
        assert int(d["delta"]) == L["delta"] and int(d["n_to_taint"]) == L["n_to_taint"], (tag, g)
        assert _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]) and _bits(d["mem_pct"]) == _bits(L["mem_pct"]), (tag, g)
        assert (int(d["cached_cpu_m"]), int(d["cached_mem_b"])) == (L["cached_cpu_m"], L["cached_mem_b"]), (tag, g)
        unt, tn = L["untainted"], L["tainted"]
        assert list(ctx.group_order(g, 0)) == \
            [idx[unt[i]] for i in O.oldest_first([lst[k]["created_ns"] for k in unt])], (tag, g)
        assert list(ctx.group_order(g, 1)) == \
            [idx[tn[i]] for i in O.newest_first([lst[k]["created_ns"] for k in tn])], (tag, g)


def esc_branch(d):
    from escalator_amd._lib import BRANCHES
    return BRANCHES[d["branch"]]


@pytest.mark.parametrize("seed", range(6))
def test_node_relabel_vs_literal(esc, seed):
    """Node Update events that change labels and creation times in place (esc_nodes_relabel,
    VERDICT r3 item 5): nodes move between groups, gain / lose extra labels and group
    memberships, change age, taint, cordon and allocatable, between node additions and
    deletions; no reload.  Totals, allNodes[0], decisions and both orderings equal the literal
    oracle on the updated nodes after every round, and a fresh age-index build agrees."""
    rng = random.Random(9900 + seed)
    G = rng.choice([3, 8, 20])
    groups = make_groups(rng, G, with_default=rng.random() < 0.6)
    pods = make_pods(rng, 300, groups, big_frac=0.0)
    nodes = make_nodes(rng, rng.choice([40, 120]), groups, big_frac=0.0)
    trackers = make_trackers(rng, groups, nodes)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    ctx.set_spare(4.0)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    if seed % 2:
        ctx.set_order_in_step(True)
    live = dict(enumerate(nodes))
    hw = len(nodes)
    _check_nodes_vs_literal(ctx, groups, states, pods, live, trackers, "load")
    in_place = 0
    for rnd in range(5):
        ids = rng.sample(sorted(live), k=min(len(live), rng.randrange(1, 10)))
        new = [_relabel(rng, live[j], groups, move_time=seed >= 2) for j in ids]
        _, packed = ctx.pack([], new)
        before = ctx.decide_all(states)[0].tobytes()
        try:
            ctx.nodes_relabel(ids, packed)
            in_place += 1
        except esc._lib.EscError as e:                   # a small group's spare room is short
            assert e.code == esc._lib.ESC_E_LIMIT
            assert ctx.decide_all(states)[0].tobytes() == before          # nothing applied
            for j, x in zip(ids, new):
                live[j] = x
            lst = [live[j] for j in sorted(live)]
            ctx.load(*ctx.pack(pods, lst, trackers))
            live = dict(enumerate(lst))
            hw = len(lst)
        else:
            for j, x in zip(ids, new):
                live[j] = x
        _check_nodes_vs_literal(ctx, groups, states, pods, live, trackers, (rnd, "relabel"))
        dels = rng.sample(sorted(live), k=min(len(live), rng.randrange(0, 4)))
        if dels:
            ctx.nodes_delete(dels)
            for j in dels:
                del live[j]
        add = make_nodes(rng, rng.randrange(0, 4), groups, big_frac=0.0)
        for k, x in enumerate(add):
            x["name"] = "r%d-add%d" % (rnd, k)
        if add:
            _, packed = ctx.pack([], add)
            try:
                got = ctx.nodes_add(packed)
            except esc._lib.EscError as e:               # spare room short: reload
                assert e.code == esc._lib.ESC_E_LIMIT
                lst = [live[j] for j in sorted(live)] + add
                ctx.load(*ctx.pack(pods, lst, trackers))
                live = dict(enumerate(lst))
                hw = len(lst)
            else:
                assert list(got) == list(range(hw, hw + len(add)))
                for j, x in zip(got, add):
                    live[int(j)] = x
                hw += len(add)
        _check_nodes_vs_literal(ctx, groups, states, pods, live, trackers, (rnd, "add/delete"))
    assert in_place >= 2, in_place
    before = {(g, w): list(ctx.group_order(g, w)) for g in range(G) for w in (0, 1)}
    ctx.build_age_index()
    ctx.sort_nodes()
    assert before == {(g, w): list(ctx.group_order(g, w)) for g in range(G) for w in (0, 1)}


def test_node_relabel_limit_all_or_nothing(esc):
    """A relabel batch whose new memberships do not fit the spare room is refused whole
    (ESC_E_LIMIT); a bad id is ESC_E_INVAL; smaller batches then apply."""
    groups = [{"name": "a", "label_key": "k", "label_value": "a", "max_nodes": 1000},
              {"name": "b", "label_key": "k", "label_value": "b", "max_nodes": 1000}]
    nodes = [{"name": "n%d" % i, "labels": {"k": "a"}, "cpu": 1000, "mem": 1000, "created_ns": i} for i in range(40)]
    nodes += [{"name": "m%d" % i, "labels": {"k": "b"}, "cpu": 10, "mem": 10, "created_ns": 100 + i} for i in range(4)]
    ctx = esc.Context(groups)
    ctx.set_spare(0.01)
    ctx.load(*ctx.pack([], nodes))
    moved = [dict(nodes[i], labels={"k": "b"}) for i in range(40)]
    _, packed = ctx.pack([], moved)
    with pytest.raises(esc._lib.EscError) as e:
        ctx.nodes_relabel(list(range(40)), packed)
    assert e.value.code == esc._lib.ESC_E_LIMIT
    tot, _ = ctx.decide_all()
    assert list(tot["n_nodes"]) == [40, 4] and list(tot["node_cpu_m"]) == [40000, 40]
    with pytest.raises(esc._lib.EscError):
        ctx.nodes_relabel([99], ctx.pack([], moved[:1])[1])
    _, packed = ctx.pack([], moved[:3])
    ctx.nodes_relabel([0, 1, 2], packed)
    tot, _ = ctx.decide_all()
    assert list(tot["n_nodes"]) == [37, 7] and list(tot["first_node"]) == [3, 0]
    assert list(tot["node_cpu_m"]) == [37000, 3040]


def test_node_relabel_churn_reuses_entries(esc):
    """Label churn (nodes moving a -> b -> a ... every round) takes each node's own retired
    entry back instead of a spare one, so 30 rounds fit a spare room of a few
    entries; the totals, allNodes[0] and both orderings stay equal to the literal oracle."""
    groups = [{"name": "a", "label_key": "k", "label_value": "a", "max_nodes": 1000},
              {"name": "b", "label_key": "k", "label_value": "b", "max_nodes": 1000}]
    nodes = [{"name": "n%d" % i, "labels": {"k": "a"}, "cpu": 1000 + i, "mem": 1000, "created_ns": i}
             for i in range(40)]
    nodes += [{"name": "m%d" % i, "labels": {"k": "b"}, "cpu": 10, "mem": 10, "created_ns": 100 + i} for i in range(4)]
    ctx = esc.Context(groups)
    ctx.set_spare(0.01)
    ctx.load(*ctx.pack([], nodes))
    live = dict(enumerate(nodes))
    movers = [0, 5, 17]
    for rnd in range(30):
        to = "b" if rnd % 2 == 0 else "a"
        new = [dict(live[j], labels={"k": to}) for j in movers]
        ctx.nodes_relabel(movers, ctx.pack([], new)[1])          # never ESC_E_LIMIT
        for j, x in zip(movers, new):
            live[j] = x
        tot, _ = ctx.decide_all()
        na = sum(1 for x in live.values() if x["labels"]["k"] == "a")
        assert list(tot["n_nodes"]) == [na, 44 - na], rnd
        assert int(tot["node_cpu_m"][0]) == sum(x["cpu"] for x in live.values() if x["labels"]["k"] == "a")
        assert int(tot["first_node"][0]) == min(j for j, x in live.items() if x["labels"]["k"] == "a")
        ctx.sort_nodes()
        for g, name in enumerate("ab"):
            mem = sorted((x["created_ns"], j) for j, x in live.items() if x["labels"]["k"] == name)
            assert list(ctx.group_order(g, 0)) == [j for _, j in mem], (rnd, g)


def test_node_add_limit_all_or_nothing(esc):
    """A batch that does not fit the spare room is refused whole (ESC_E_LIMIT)."""
    groups = [{"name": "a", "label_key": "k", "label_value": "v", "max_nodes": 1000}]
    nodes = [{"name": "n%d" % i, "labels": {"k": "v"}, "cpu": 1000, "mem": 1000, "created_ns": i} for i in range(8)]
    ctx = esc.Context(groups)
    ctx.set_spare(0.01)
    ctx.load(*ctx.pack([], nodes))
    more = [{"name": "m%d" % i, "labels": {"k": "v"}, "cpu": 1, "mem": 1, "created_ns": 100 + i} for i in range(64)]
    _, packed = ctx.pack([], more)
    with pytest.raises(esc._lib.EscError):
        ctx.nodes_add(packed)
    tot, _ = ctx.decide_all()
    assert tot["n_nodes"][0] == 8 and tot["node_cpu_m"][0] == 8000
    _, packed = ctx.pack([], more[:3])
    assert list(ctx.nodes_add(packed)) == [8, 9, 10]
    tot, _ = ctx.decide_all()
    assert tot["n_nodes"][0] == 11 and tot["node_cpu_m"][0] == 8003


def _members_oldest(nodes, groups, g):
    """All members of dry group g, oldest first (ties by index): the oracle's two lists merged."""
    both = list(soa.order(nodes, groups, g, 0)) + list(soa.order(nodes, groups, g, 1))
    t = nodes["created_ns"]
    return sorted(both, key=lambda j: (int(t[j]), j))


@pytest.mark.parametrize("graph", [False, True])
def test_sharded_two_contexts_host_exchange(esc, graph):
    """Three ranks' shards on one device, exchanged through the host: == whole snapshot
    (graph: each shard's K1/K2/K3 step replayed from its captured graph, twice); each rank
    decides the groups it owns and the owners' records make up every group."""
    from escalator_amd.dist import merge_owned, merge_owned_metrics, shard_range
    P, N, G = 300_000, 30_000, 1000
    full = esc.Synth(P, N, G, config=4, seed=11)
    otot = soa.totals(full.pods(), full.nodes(), full.groups)
    odf, odi = soa.decide(full.groups, full.states, otot)
    ctxs, words, firsts = [], [], []
    for r in range(3):
        lo, hi = shard_range(P, r, 3)
        s = esc.Synth(P, N, G, config=4, seed=11, p_lo=lo, p_hi=hi)
        c = esc.Context(s, rank=r, world=3)
        c.load_synth(s, pod_offset=lo)
        c.set_state(full.states)
        c.use_graph(graph)
        for _ in range(2 if graph else 1):
            c.reduce()
        w, f = c.exchange_download()
        words.append(w)
        firsts.append(f)
        ctxs.append((c, s))
    W = np.sum(words, axis=0)
    F = np.min(firsts, axis=0)
    parts, mets = [], []
    for c, _ in ctxs:
        c.set_metrics(True)
        c.exchange_upload(W, F)
        c.decide()
        parts.append(c.results())                # each rank: its own groups
        mets.append(c.metrics())
    tot, dec = merge_owned(parts)
    check_against_c_oracle(tot, dec, otot, odf, odi)
    owners = [ctxs[0][0].group_owner(g) for g in range(G)]
    assert set(owners) == {0, 1, 2}
    check_metrics(merge_owned_metrics(mets, owners), soa.metrics(otot, odf, odi))


def test_determinism_repeat(esc):
    s = esc.Synth(500_000, 5_000, 500, config=4, seed=99)
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    ctx.run()
    t0, d0 = ctx.results()
    for _ in range(5):
        ctx.run()
        t1, d1 = ctx.results()
        assert t0.tobytes() == t1.tobytes() and d0.tobytes() == d1.tobytes()


def test_big_tiles_and_window_edges(esc):
    """Tiles with > 128 extra records (k_pod_bigtiles) and pods spilled to the wide path."""
    groups = [{"name": "g%d" % i, "label_key": "k", "label_value": "v%d" % i, "max_nodes": 1000} for i in range(5)]
    rng = random.Random(9)
    pods = []
    for i in range(1100):
        n_c = 9 if 256 <= i < 512 else rng.choice([1, 2])          # tile 1 overflows the register chunks
        sel = {"k": "v%d" % rng.randrange(5)}
        expr = {"key": "k", "op": "In", "values": ["v%d" % j for j in range(5)]}
        aff = {"node_affinity": {"required": [[expr]]}, "pod_affinity": False,
               "pod_anti_affinity": False} if 600 <= i < 900 else None
        pods.append({"containers": [{"cpu": rng.randrange(1, 5000), "mem": rng.randrange(1, 1 << 36)}
                                    for _ in range(n_c)],
                     "init_containers": [{"cpu": rng.randrange(1, 9000), "mem": None}] if i % 7 == 0 else [],
                     "overhead": {"cpu": 7, "mem": 11} if i % 5 == 0 else None,
                     "node_selector": sel, "affinity": aff})
    nodes = [{"name": "n%d" % i, "labels": {"k": "v%d" % (i % 5)}, "cpu": 4000, "mem": 8 << 30,
              "created_ns": i} for i in range(40)]
    ctx = esc.Context(groups)
    P, N = ctx.pack(pods, nodes)
    ctx.load(P, N)
    tot, dec = ctx.decide_all()
    otot = soa.totals(P, N, groups)
    odf, odi = soa.decide(groups, None, otot)
    check_against_c_oracle(tot, dec, otot, odf, odi)
    for g in range(5):
        L = O.scale_node_group(groups[g], {}, pods, nodes)
        assert (tot["pod_cpu_m"][g], tot["pod_mem_b"][g], tot["n_pods"][g]) == (L["pod_cpu_m"], L["pod_mem_b"], L["n_pods"])


def test_node_sums_value_ranges(esc):
    """K2's two accumulation paths: allocatable in [0, 2^54) summed whole (one word per
    sum), anything else (negative, >= 2^54) split in lo32 / hi parts — in the same piece and
    the same wave-load as small ones, up to 2^54 - 1 x 1 024 members (the small path's
    bound), and past int64 (the node-overflow flag) — against the C oracle and the literal
    one's totals."""
    rng = random.Random(54)
    groups = [{"name": "g%d" % i, "label_key": "k", "label_value": "v%d" % i, "max_nodes": 100000}
              for i in range(7)]
    nodes, j = [], 0

    def add(g, cpu, mem, n):
        nonlocal j
        for _ in range(n):
            nodes.append({"name": "n%d" % j, "labels": {"k": "v%d" % g}, "cpu": cpu() if callable(cpu) else cpu,
                          "mem": mem() if callable(mem) else mem, "created_ns": j,
                          "unschedulable": rng.random() < 0.1})
            j += 1

    add(0, (1 << 54) - 1, (1 << 54) - 1, 1024)                  # the small path at its bound: LO near 2^64, int64 overflow
    add(6, 1 << 53, (1 << 53) - 1, 1023)                        # large, whole, still inside int64
    add(1, lambda: rng.choice([5, 1 << 54, -3]), lambda: rng.choice([7, 1 << 60, -(1 << 40)]), 700)  # mixed
    add(2, 1 << 62, 1 << 62, 5)                                 # past int64: flagged
    add(3, lambda: rng.randrange(0, 1 << 20), lambda: rng.randrange(0, 1 << 40), 2000)   # typical
    add(4, -1, -(1 << 63), 3)                                   # negative extremes
    add(5, lambda: rng.randrange(-(1 << 63), 1 << 63), lambda: rng.randrange(-(1 << 63), 1 << 63), 300)
    ctx = esc.Context(groups)
    P, N = ctx.pack([], nodes)
    ctx.load(P, N)
    tot, dec = ctx.decide_all()
    otot = soa.totals(P, N, groups)
    odf, odi = soa.decide(groups, None, otot)
    check_against_c_oracle(tot, dec, otot, odf, odi)
    assert tot["flags"][0] != 0 and tot["flags"][2] != 0 and tot["flags"][3] == 0 and tot["flags"][6] == 0
    unt6 = [x for x in nodes if x["labels"]["k"] == "v6" and not x["unschedulable"]]
    assert (tot["node_cpu_m"][6], tot["node_mem_b"][6]) == (sum(x["cpu"] for x in unt6), sum(x["mem"] for x in unt6))


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_node_index_split_within_pairs(esc, world):
    """Pairs with many pieces (10k members each), a dry group with tracked members, the
    node index split across `world` ranks inside pairs; SUM of the ranks' words == the
    whole snapshot, and every rank resolves allNodes[0] on its own."""
    from escalator_amd import layout
    from oracle import soa as S
    P, N, G = 50_000, 200_000, 20
    full = esc.Synth(P, N, G, config=5, seed=0xE5CA1A7E00000005)
    assert any(g.get("dry_mode") for g in full.groups) and len(full.nodes()["trk_node"]) > 0
    otot = S.totals(full.pods(), full.nodes(), full.groups)
    odf, odi = S.decide(full.groups, full.states, otot)
    ctxs, words = [], []
    n_gp = len(S.group_tables(full.groups)["pair_ids"])
    for r in range(world):
        from escalator_amd.dist import shard_range
        lo, hi = shard_range(P, r, world)
        s = esc.Synth(P, N, G, config=5, seed=0xE5CA1A7E00000005, p_lo=lo, p_hi=hi)
        c = esc.Context(s, rank=r, world=world)
        c.load_synth(s, pod_offset=lo)
        pb, nb = c.stream_bytes()
        assert pb == layout.pod_bytes(s.pods(), n_gp)
        assert nb == layout.node_bytes(s.nodes(), n_gp, r, world)
        c.set_state(full.states)
        c.reduce()
        w, m = c.exchange_download()
        assert m.size == 0
        words.append(w)
        ctxs.append((c, s))
    W = np.sum(words, axis=0)
    parts = []
    for c, _ in ctxs:
        c.exchange_upload(W, np.zeros(0, np.int64))
        c.decide()
        parts.append(c.results())
    from escalator_amd.dist import merge_owned
    tot, dec = merge_owned(parts)
    check_against_c_oracle(tot, dec, otot, odf, odi)


# ------------------------------------------------- incremental snapshot (§8f)
def _packed_subset(P: dict, idx: list[int]) -> dict:
    """The packed records of pods `idx` (in that order) out of a `pack` result."""
    from escalator_amd.layout import NONE  # noqa: F401
    f = P["flags"].astype(np.uint64)
    nxc = ((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1)
    nxp = (f >> 24) & 0x3F
    oc = np.concatenate([[0], np.cumsum(nxc)]).astype(np.int64)
    op = np.concatenate([[0], np.cumsum(nxp)]).astype(np.int64)
    out = {k: P[k][idx] for k in ("flags", "cpu0", "mem0", "pair0")}
    out["xc_cpu"] = np.concatenate([P["xc_cpu"][oc[i]:oc[i + 1]] for i in idx] or [np.zeros(0, np.int64)])
    out["xc_mem"] = np.concatenate([P["xc_mem"][oc[i]:oc[i + 1]] for i in idx] or [np.zeros(0, np.int64)])
    out["xp_pair"] = np.concatenate([P["xp_pair"][op[i]:op[i + 1]] for i in idx] or [np.zeros(0, np.uint32)])
    return out


def _fits_k(P: dict, i: int) -> bool:
    f = int(P["flags"][i])
    return ((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1) <= 3 and ((f >> 24) & 0x3F) <= 3


@pytest.mark.parametrize("seed", range(4))
def test_incremental_events_vs_literal(esc, seed):
    """Pod upserts / deletes / inserts and node taint / cordon / allocatable events patch the
    resident snapshot (esc_pods_upsert, esc_pods_delete, esc_nodes_update); every decision
    and ordering then equals the literal oracle on the updated object lists."""
    from escalator_amd._lib import ESC_E_LIMIT
    rng = random.Random(7000 + seed)
    G = rng.choice([3, 8])
    groups = make_groups(rng, G, with_default=True)
    pods = make_pods(rng, 400, groups, big_frac=0.0)
    nodes = make_nodes(rng, 60, groups, big_frac=0.0)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    ctx.set_spare(0.5)
    P, N = ctx.pack(pods, nodes)
    ctx.load(P, N)
    live = {i: p for i, p in enumerate(pods)}
    next_id = len(pods)
    for rnd in range(3):
        # pod events: deletes, in-place changes, inserts (only shapes the K layout holds)
        ev_ids, ev_objs = [], []
        for i in rng.sample(sorted(live), 30):
            q = make_pods(rng, 1, groups, big_frac=0.0)[0]
            ev_ids.append(i)
            ev_objs.append(q)
        for _ in range(20):
            ev_ids.append(next_id)
            ev_objs.append(make_pods(rng, 1, groups, big_frac=0.0)[0])
            next_id += 1
        Pe, _ = ctx.pack(ev_objs, [])
        keep = [k for k in range(len(ev_ids)) if _fits_k(Pe, k)]
        rc = ctx.pods_upsert([ev_ids[k] for k in keep], _packed_subset(Pe, keep))
        assert rc == 0, rc
        for k in keep:
            live[ev_ids[k]] = ev_objs[k]
        dels = rng.sample(sorted(live), 25)
        ctx.pods_delete(dels)
        for i in dels:
            del live[i]
        # node events: taint / cordon / allocatable
        nid = rng.sample(range(len(nodes)), 12)
        for j in nid:
            nd = nodes[j]
            nd["unschedulable"] = rng.random() < 0.3
            nd["taints"] = ["atlassian.com/escalator"] if rng.random() < 0.4 else []
            nd["cpu"] = rng.choice([0, 2000, 4000, 16000])
            nd["mem"] = rng.choice([0, 8 << 30, 64 << 30])
        _, Nn = ctx.pack([], nodes)
        ctx.nodes_update(nid, Nn["flags"][nid], Nn["cpu"][nid], Nn["mem"][nid])
        # decisions and orderings vs the literal oracle over the live objects
        cur = [live[i] for i in sorted(live)]
        tot, dec = ctx.decide_all(states)
        ctx.sort_nodes()
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], cur, nodes)
            t, d = tot[g], dec[g]
            assert (t["n_pods"], t["n_nodes"], t["n_untainted"], t["n_tainted"], t["n_cordoned"]) == \
                (L["n_pods"], L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"]), (rnd, g)
            assert (t["pod_cpu_m"], t["pod_mem_b"], t["node_cpu_m"], t["node_mem_b"]) == \
                (L["pod_cpu_m"], L["pod_mem_b"], L["node_cpu_m"], L["node_mem_b"]), (rnd, g)
            assert int(d["delta"]) == L["delta"] and _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]), (rnd, g)
            assert (int(d["cached_cpu_m"]), int(d["cached_mem_b"])) == (L["cached_cpu_m"], L["cached_mem_b"])
            unt = L["untainted"]
            assert list(ctx.group_order(g, 0)) == [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
    # more inserts than the spare holds: refused whole, nothing applied
    many = make_pods(rng, 2000, groups, big_frac=0.0)
    Pm, _ = ctx.pack(many, [])
    keep = [k for k in range(len(many)) if _fits_k(Pm, k)]
    before = ctx.decide_all(states)[0].tobytes()
    assert ctx.pods_upsert([next_id + k for k in range(len(keep))], _packed_subset(Pm, keep)) == ESC_E_LIMIT
    assert ctx.decide_all(states)[0].tobytes() == before


@pytest.mark.parametrize("seed", range(3))
def test_k_block_formats_vs_literal(esc, seed):
    """Pods at the edges of the three K block formats (plain; packed: cpu < 2^20 - 1, mem <
    2^44 - 1; packed small: first container cpu < 2^14, mem < 2^34) and init containers with
    absent keys, through the layout and upserts that move pods between formats: totals and
    decisions equal the literal oracle, and esc_stream_bytes the restated format bytes."""
    from escalator_amd import layout
    from randobj import _req
    rng = random.Random(7600 + seed)
    G = rng.choice([3, 12])
    groups = make_groups(rng, G, with_default=True)
    edges_c = [0, 1, (1 << 14) - 1, 1 << 14, (1 << 20) - 2, (1 << 20) - 1, -1, None]
    edges_m = [0, 1, (1 << 34) - 1, 1 << 34, (1 << 44) - 2, (1 << 44) - 1, -1, None]

    def edge_pod():
        q = make_pods(rng, 1, groups, big_frac=0.0)[0]
        reqs = q["containers"] + q["init_containers"]
        for r in reqs:
            if rng.random() < 0.5:
                r["cpu"] = rng.choice(edges_c)
            if rng.random() < 0.5:
                r["mem"] = rng.choice(edges_m)
        return q

    pods = [edge_pod() for _ in range(400)]
    nodes = make_nodes(rng, 40, groups, big_frac=0.0)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    ctx.set_spare(1.0)
    P, N = ctx.pack(pods, nodes)
    ctx.load(P, N)
    n_gp = ctx.lib.esc_ctx_num_group_pairs(ctx.handle)
    live = dict(enumerate(pods))
    for rnd in range(3):
        if rnd:
            ids = rng.sample(sorted(live), 60)
            objs = [edge_pod() for _ in ids]
            Pe, _ = ctx.pack(objs, [])
            assert ctx.pods_upsert(ids, Pe) == 0
            for i, q in zip(ids, objs):
                live[i] = q
        cur = [live[i] for i in sorted(live)]
        tot, dec = ctx.decide_all(states)
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], cur, nodes)
            t, d = tot[g], dec[g]
            assert t["n_pods"] == L["n_pods"], (rnd, g)
            if L["pod_cpu_m"] is not None:
                assert (t["pod_cpu_m"], t["pod_mem_b"]) == (L["pod_cpu_m"], L["pod_mem_b"]), (rnd, g)
            assert esc._lib.BRANCHES[d["branch"]] == L["branch"], (rnd, g)
            assert int(d["delta"]) == L["delta"] and _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]), (rnd, g)
        if rnd == 0:
            assert ctx.stream_bytes()[0] == layout.pod_bytes(P, n_gp)


@pytest.mark.parametrize("seed", range(4))
def test_c_pod_events_vs_literal(esc, seed):
    """Upserts of pods outside the K classes (more than 3 extra container records: the C
    section) patch in place (§8f rank 1): into the pod's own C slot when it has room, else
    into a spare C slot (esc_set_spare), whose unused records stay neutral; pods change
    between the K and C sections, are deleted and re-inserted.  Every decision then equals
    the literal oracle; a pod bigger than any free slot's room is refused whole."""
    from escalator_amd._lib import ESC_E_LIMIT
    from randobj import _req
    rng = random.Random(7300 + seed)
    G = rng.choice([3, 8])
    groups = make_groups(rng, G, with_default=True)

    def c_pod(n_reg=5):                      # 5 containers (4 extra records, + init / overhead): a C pod
        q = make_pods(rng, 1, groups, big_frac=0.0)[0]
        # (a first container with a negative cpu is not inline: 5 extra records, more than a
        # spare slot's room, so big values only from the second one on)
        q["containers"] = [_req(rng, k > 0 and rng.random() < 0.05) for k in range(n_reg)]
        return q

    pods = make_pods(rng, 300, groups, big_frac=0.02) + [c_pod() for _ in range(40)]
    nodes = make_nodes(rng, 60, groups, big_frac=0.0)
    states = make_states(rng, G)
    ctx = esc.Context(groups)
    ctx.set_spare(2.0)                       # spare C room: max(16, 2 x 40) slots
    P, N = ctx.pack(pods, nodes)
    assert sum(not _fits_k(P, k) for k in range(len(pods))) >= 40
    ctx.load(P, N)
    live = dict(enumerate(pods))
    next_id = len(pods)
    for rnd in range(3):
        ev_ids, ev_objs = [], []
        for i in rng.sample(sorted(live), 16):               # K <-> C changes of existing pods
            ev_ids.append(i)
            ev_objs.append(c_pod() if rng.random() < 0.6 else make_pods(rng, 1, groups, big_frac=0.02)[0])
        for _ in range(6):                                   # new C pods
            ev_ids.append(next_id)
            ev_objs.append(c_pod())
            next_id += 1
        Pe, _ = ctx.pack(ev_objs, [])
        assert ctx.pods_upsert(ev_ids, Pe) == 0, rnd
        for i, q in zip(ev_ids, ev_objs):
            live[i] = q
        dels = rng.sample(sorted(live), 12)
        ctx.pods_delete(dels)
        for i in dels:
            del live[i]
        cur = [live[i] for i in sorted(live)]
        tot, dec = ctx.decide_all(states)
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], cur, nodes)
            t, d = tot[g], dec[g]
            assert t["n_pods"] == L["n_pods"], (rnd, g)
            assert (t["pod_cpu_m"], t["pod_mem_b"]) == (L["pod_cpu_m"], L["pod_mem_b"]) or L["pod_cpu_m"] is None, (rnd, g)
            assert esc._lib.BRANCHES[d["branch"]] == L["branch"], (rnd, g)
            assert int(d["delta"]) == L["delta"] and _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]), (rnd, g)
    # a pod with more containers than any free C slot holds: nothing applied
    before = ctx.decide_all(states)[0].tobytes()
    Pb, _ = ctx.pack([c_pod(9)], [])
    assert ctx.pods_upsert([next_id], Pb) == ESC_E_LIMIT
    assert ctx.decide_all(states)[0].tobytes() == before


# ------------------------------------------------ scale-down reaping (§8f rank 2)
def _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, soft, hard):
    res = ctx.try_remove(now_ns, soft, hard)
    for g, grp in enumerate(groups):
        L = O.scale_node_group(grp, {}, pods, nodes, tracker=trackers.get(g, []))
        pods_g = O.filtered_list(pods, O.group_pod_filter(grp))
        all_nodes = [nodes[i] for i in range(len(nodes))
                     if O.new_node_label_filter_func(grp.get("label_key", ""), grp.get("label_value", ""))(nodes[i])]
        tainted = L["tainted"]
        neg, remaining, ks = O.try_remove_tainted_nodes(grp, [nodes[i] for i in tainted], pods_g, all_nodes,
                                                        now_ns, int(soft[g]), int(hard[g]), bool(grp.get("dry_mode")))
        r = res[g]
        assert int(r["n_candidates"]) == len(tainted), g
        assert (-int(r["n_delete"]), int(r["pods_remaining"])) == (neg, remaining), (g, neg, remaining)
        assert list(ctx.removal_nodes(g)) == [tainted[k] for k in ks], g


@pytest.mark.parametrize("seed", range(6))
def test_try_remove_tainted_vs_literal(esc, seed):
    """TryRemoveTaintedNodes for every group at once (esc_load_placement + esc_try_remove):
    deletion lists, counts and NodePodsRemaining sums equal the literal oracle, including
    no-delete annotations, unparsable taint values, dry-mode groups, pods bound to no /
    unknown nodes and nodes shared by several groups; a pod delete keeps the binding."""
    from escalator_amd.objects import placement
    rng = random.Random(9100 + seed)
    G = rng.choice([1, 4, 12])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, rng.choice([0, 300, 1500]), rng.choice([5, 60, 200]))
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    P, N = ctx.pack(pods, nodes, trackers)
    assert len(P["flags"]) == len(pods)
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(pn, ts, nd)
    for _ in range(3):
        soft = np.array([rng.choice([0, 60, 300, 600]) * 10**9 for _ in range(G)], np.int64)
        hard = soft + np.array([rng.choice([0, 120, 600]) * 10**9 for _ in range(G)], np.int64)
        _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, soft, hard)
    # node facts refreshed without re-binding pods
    for x in rng.sample(nodes, min(len(nodes), 5)):
        x["taint_value"] = str(now_ns // 10**9 - 5000)
        x["annotations"] = {}
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(None, ts, nd)
    _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, np.full(G, 60 * 10**9), np.full(G, 4000 * 10**9))
    if pods:                                      # a pod event keeps the binding current
        ctx.pods_delete([0])
        del pods[0]
        _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, np.full(G, 60 * 10**9), np.full(G, 4000 * 10**9))


@pytest.mark.parametrize("seed", range(5))
def test_reaping_follows_pod_events(esc, seed):
    """The placement survives pod events (§8f rank 2): upserts rewrite a bound pod's
    reference (its record and slot may change), deletes drop it, esc_pods_bind moves pods
    between nodes / binds new pods; TryRemoveTaintedNodes then equals the literal oracle on
    the live pods with their current Spec.NodeName."""
    from escalator_amd.objects import placement
    rng = random.Random(9300 + seed)
    G = rng.choice([2, 6, 12])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 600, rng.choice([20, 80]))
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    ctx.set_spare(0.5)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(pn, ts, nd)
    index = {n["name"]: j for j, n in enumerate(nodes)}
    live = dict(enumerate(pods))
    next_id = len(pods)
    soft = np.array([rng.choice([0, 60, 300]) * 10**9 for _ in range(G)], np.int64)
    hard = soft + np.array([rng.choice([0, 600]) * 10**9 for _ in range(G)], np.int64)
    for rnd in range(4):
        # upserts of existing pods (new records; some move node) and inserts of new pods
        ev_ids, ev_objs = [], []
        for i in rng.sample(sorted(live), min(len(live), 40)):
            q = make_pods(rng, 1, groups, big_frac=0.0)[0]
            q["node_name"] = live[i]["node_name"] if rng.random() < 0.7 else rng.choice(nodes)["name"]
            ev_ids.append(i)
            ev_objs.append(q)
        for _ in range(25):
            q = make_pods(rng, 1, groups, big_frac=0.0)[0]
            q["node_name"] = rng.choice(nodes)["name"] if rng.random() < 0.8 else ""
            ev_ids.append(next_id)
            ev_objs.append(q)
            next_id += 1
        Pe, _ = ctx.pack(ev_objs, [])
        keep = [k for k in range(len(ev_ids)) if _fits_k(Pe, k)]
        assert ctx.pods_upsert([ev_ids[k] for k in keep], _packed_subset(Pe, keep)) == 0
        bind_ids, bind_to = [], []
        for k in keep:
            i, q = ev_ids[k], ev_objs[k]
            old = live[i]["node_name"] if i in live else ""
            live[i] = q
            if q["node_name"] != old:
                bind_ids.append(i)
                bind_to.append(index.get(q["node_name"], 0xFFFFFFFF) if q["node_name"] else 0xFFFFFFFF)
        def bind(ids_, to_):
            try:
                ctx.pods_bind(ids_, to_)
            except esc._lib.EscError as e:            # a node's run is full: re-bind everything
                assert e.code == esc._lib.ESC_E_LIMIT
                full = np.full(next_id, 0xFFFFFFFF, np.uint32)
                for i_, t_ in zip(ids_, to_):
                    live[i_] = dict(live[i_], node_name=nodes[t_]["name"] if t_ != 0xFFFFFFFF else "")
                for i_, q_ in live.items():
                    if q_.get("node_name") in index:
                        full[i_] = index[q_["node_name"]]
                ctx.load_placement(full, ts, nd)

        if bind_ids:
            bind(bind_ids, bind_to)
        dels = rng.sample(sorted(live), 30)
        ctx.pods_delete(dels)
        for i in dels:
            del live[i]
        # pods rescheduled to other nodes (or unbound) without a record change
        mv = rng.sample(sorted(live), 20)
        to = [rng.choice(nodes)["name"] if rng.random() < 0.85 else "" for _ in mv]
        bind(mv, [index[t] if t else 0xFFFFFFFF for t in to])
        for i, t in zip(mv, to):
            live[i] = dict(live[i], node_name=t)
        cur = [live[i] for i in sorted(live)]
        _check_reaping(ctx, groups, cur, nodes, trackers, now_ns, soft, hard)


def _many_pair_pod(rng, groups, node_name):
    """A pod outside the K classes by its pairs: one node-affinity `In` term over 5-7 values
    of one group key (4-6 extra pairs: > 3, so its PodRef reads them through its xp offset;
    <= 6, a spare C slot's room)."""
    q = make_pods(rng, 1, groups, big_frac=0.0)[0]
    keyed = [g for g in groups if g["label_key"]]
    k = rng.choice(keyed)["label_key"] if keyed else "customer"
    vals = sorted({g["label_value"] for g in groups if g["label_key"] == k} | {"x%d" % i for i in range(9)})
    rng.shuffle(vals)
    q["node_selector"] = None
    q["owner_kinds"] = []
    q["affinity"] = {"node_affinity": {"required": [[{"key": k, "op": "In", "values": vals[:rng.randrange(5, 8)]}]]},
                     "pod_affinity": False, "pod_anti_affinity": False}
    q["node_name"] = node_name
    return q


@pytest.mark.parametrize("seed", range(4))
def test_reaping_follows_c_pod_upserts(esc, seed):
    """upserts of BOUND pods with more than 3 extra pairs (C section, indirect
    PodRefs) whose pairs change, K <-> C moves and C-slot reuse inside one batch: the node
    occupancy words follow (the old contribution leaves before the record is patched), so
    TryRemoveTaintedNodes equals the literal oracle on the live pods."""
    from escalator_amd.objects import placement
    rng = random.Random(9700 + seed)
    G = rng.choice([4, 8])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 300, 30)
    pods += [_many_pair_pod(rng, groups, rng.choice(nodes)["name"]) for _ in range(60)]
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    ctx.set_spare(2.0)
    P, N = ctx.pack(pods, nodes, trackers)
    assert sum(not _fits_k(P, k) for k in range(len(pods))) >= 60
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(pn, ts, nd)
    live = dict(enumerate(pods))
    soft = np.full(G, 60 * 10**9, np.int64)
    hard = np.full(G, 4000 * 10**9, np.int64)
    _check_reaping(ctx, groups, [live[i] for i in sorted(live)], nodes, trackers, now_ns, soft, hard)
    for rnd in range(4):
        bound = [i for i in sorted(live) if live[i]["node_name"] and not _fits_k(P, i)]
        ev_ids, ev_objs = [], []
        for i in rng.sample(bound, min(len(bound), 20)):       # C pods: new pairs (or into K), same node
            q = _many_pair_pod(rng, groups, live[i]["node_name"]) if rng.random() < 0.7 else \
                dict(make_pods(rng, 1, groups, big_frac=0.0)[0], node_name=live[i]["node_name"])
            ev_ids.append(i)
            ev_objs.append(q)
        kb = [i for i in sorted(live) if live[i]["node_name"] and i not in ev_ids]
        for i in rng.sample(kb, min(len(kb), 10)):             # K pods into C (may reuse a slot freed above)
            ev_ids.append(i)
            ev_objs.append(_many_pair_pod(rng, groups, live[i]["node_name"]))
        Pe, _ = ctx.pack(ev_objs, [])
        assert ctx.pods_upsert(ev_ids, Pe) == 0, rnd
        for i, q in zip(ev_ids, ev_objs):
            live[i] = q
        P, _ = ctx.pack([live[i] for i in range(len(pods))], [])     # which ids are C pods now
        _check_reaping(ctx, groups, [live[i] for i in sorted(live)], nodes, trackers, now_ns, soft, hard)


@pytest.mark.parametrize("seed", range(4))
def test_reaping_across_node_relabels(esc, seed):
    """TryRemoveTaintedNodes after node relabels (esc_nodes_relabel): a relabelled node's
    pods leave the occupancy of the group pairs it no longer carries and count for the ones
    it now carries, with no placement reload (the taint facts are refreshed, not the
    binding); deletions equal the literal oracle, in snapshot order."""
    from escalator_amd.objects import placement
    rng = random.Random(9950 + seed)
    G = rng.choice([4, 8])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 800, 60)
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    ctx.set_spare(4.0)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(pn, ts, nd)
    soft = np.full(G, 60 * 10**9, np.int64)
    hard = np.full(G, 4000 * 10**9, np.int64)
    for rnd in range(4):
        ids = rng.sample(range(len(nodes)), 6)
        new = []
        for j in ids:
            x = _relabel(rng, nodes[j], groups, move_time=rnd % 2 == 1)
            x["taint_value"] = nodes[j].get("taint_value")
            if rng.random() < 0.5 and "atlassian.com/escalator" not in x["taints"]:
                x["taints"] = x["taints"] + ["atlassian.com/escalator"]
            new.append(x)
        _, packed = ctx.pack([], new)
        ctx.nodes_relabel(ids, packed)
        for j, x in zip(ids, new):
            nodes[j] = x
        _, ts, nd = placement(pods, nodes)
        ctx.load_placement(None, ts, nd)                   # the node facts (taint times) only
        _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, soft, hard)


@pytest.mark.parametrize("seed", range(4))
def test_reaping_across_node_events(esc, seed):
    """The placement survives node informer events (§8f rank 2): node deletes, node adds
    (their pods bound with esc_pods_bind into the runs reserved for new table slots), pod
    moves and a node-facts refresh, with no esc_load_placement of the pods in between;
    TryRemoveTaintedNodes equals the literal oracle on the live nodes in snapshot order."""
    from escalator_amd.objects import placement, taint_time, NO_DELETE_ANNOTATION
    NONE = 0xFFFFFFFF
    rng = random.Random(9500 + seed)
    G = rng.choice([2, 6, 12])
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 500, rng.choice([30, 90]))
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    ctx.set_spare(2.0)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    ctx.load_placement(pn, ts, nd)
    live = dict(enumerate(nodes))
    index = {x["name"]: j for j, x in live.items()}
    pod_live = dict(enumerate(pods))
    soft = np.array([rng.choice([0, 60, 300]) * 10**9 for _ in range(G)], np.int64)
    hard = soft + np.array([rng.choice([0, 600]) * 10**9 for _ in range(G)], np.int64)
    now_s = now_ns // 10**9
    reloads = []
    hw = len(nodes)                                          # table slots in use (deleted included)
    for rnd in range(5):
        dels = rng.sample(sorted(live), k=min(len(live) - 1, rng.randrange(0, 6)))
        if dels:
            ctx.nodes_delete(dels)
            for j in dels:
                del index[live.pop(j)["name"]]
        new = make_nodes(rng, rng.randrange(1, 8), groups, big_frac=0.0)
        for k, x in enumerate(new):
            x["name"] = "r%d-new%d" % (rnd, k)
            if rng.random() < 0.6 and "atlassian.com/escalator" not in x["taints"]:
                x["taints"] = x["taints"] + ["atlassian.com/escalator"]
            x["taint_value"] = rng.choice([str(now_s - rng.randrange(0, 900)), "bad", None])
            if rng.random() < 0.15:
                x["annotations"] = {NO_DELETE_ANNOTATION: "true"}
        _, packed = ctx.pack([], new)
        try:
            ids = [int(j) for j in ctx.nodes_add(packed)]
        except esc._lib.EscError as e:                       # spare room short: reload all
            assert e.code == esc._lib.ESC_E_LIMIT
            order = sorted(live)
            lst = [live[j] for j in order] + new
            P, N = ctx.pack([pod_live[i] for i in sorted(pod_live)], lst, trackers)
            ctx.load(P, N)
            pod_live = dict(enumerate(pod_live[i] for i in sorted(pod_live)))
            live = dict(enumerate(lst))
            index = {x["name"]: j for j, x in live.items()}
            ctx.load_placement(*placement([pod_live[i] for i in sorted(pod_live)], lst))
            hw = len(lst)
            reloads.append(("nodes_add", rnd))
        else:
            assert ids == list(range(hw, hw + len(new)))
            hw += len(new)
            for j, x in zip(ids, new):
                live[j] = x
                index[x["name"]] = j
        # pods rescheduled: about the mean pods per node onto each new node (round robin),
        # others onto existing nodes or unbound
        names = [x["name"] for x in new if x["name"] in index]
        mv = rng.sample(sorted(pod_live), 6 * len(names) + 20)
        to = [names[k % len(names)] if k < 6 * len(names) else
              (live[rng.choice(sorted(live))]["name"] if rng.random() < 0.85 else "") for k in range(len(mv))]
        try:
            ctx.pods_bind(mv, [index[t] if t else NONE for t in to])
        except esc._lib.EscError as e:                       # a run is full: re-bind everything
            assert e.code == esc._lib.ESC_E_LIMIT
            for i, t in zip(mv, to):
                pod_live[i] = dict(pod_live[i], node_name=t)
            full = np.full(max(pod_live) + 1, NONE, np.uint32)
            for i, q in pod_live.items():
                full[i] = index.get(q.get("node_name") or "", NONE)
            ctx.load_placement(full, *_facts(live, hw, taint_time))
            reloads.append(("pods_bind", rnd))
        for i, t in zip(mv, to):
            pod_live[i] = dict(pod_live[i], node_name=t)
        # the node facts (taint times, no-delete) of every table slot, the new nodes' included
        ctx.load_placement(None, *_facts(live, hw, taint_time))
        idx = sorted(live)
        lst = [live[j] for j in idx]
        cur = [pod_live[i] for i in sorted(pod_live)]
        res = ctx.try_remove(now_ns, soft, hard)
        for g, grp in enumerate(groups):
            L = O.scale_node_group(grp, {}, cur, lst, tracker=trackers.get(g, []))
            pods_g = O.filtered_list(cur, O.group_pod_filter(grp))
            all_nodes = [x for x in lst if O.new_node_label_filter_func(grp.get("label_key", ""),
                                                                        grp.get("label_value", ""))(x)]
            tainted = L["tainted"]
            neg, remaining, ks = O.try_remove_tainted_nodes(grp, [lst[i] for i in tainted], pods_g, all_nodes, now_ns,
                                                            int(soft[g]), int(hard[g]), bool(grp.get("dry_mode")))
            r = res[g]
            assert int(r["n_candidates"]) == len(tainted), (rnd, g)
            assert (-int(r["n_delete"]), int(r["pods_remaining"])) == (neg, remaining), (rnd, g)
            assert list(ctx.removal_nodes(g)) == [idx[tainted[k]] for k in ks], (rnd, g)
    assert not reloads, reloads


def _facts(live, hw, taint_time):
    """esc_load_placement's node facts over table slots [0, hw) (deleted slots: none)."""
    from escalator_amd.objects import NO_DELETE_ANNOTATION
    ts = np.full(hw, np.iinfo(np.int64).min, np.int64)
    nd = np.zeros(hw, np.uint8)
    for j, x in live.items():
        ts[j] = taint_time(x)
        nd[j] = 1 if (x.get("annotations") or {}).get(NO_DELETE_ANNOTATION, "") else 0
    return ts, nd


@pytest.mark.parametrize("graphless", [True])
def test_reaping_sharded_host_exchange(esc, graphless):
    """Reaping over three pod shards on one device: each rank's K6 counts its own pods per
    tainted node, the occupancy words are summed through the host (esc_reap_download /
    _upload — the sum RCCL does in esc_try_remove), and every rank's K7 gives the
    single-context deletions (and the literal oracle's)."""
    from escalator_amd.dist import shard_range
    from escalator_amd.objects import placement
    rng = random.Random(9400)
    G = 8
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 1500, 120)
    trackers = make_trackers(rng, groups, nodes)
    pn, ts, nd = placement(pods, nodes)
    soft = np.full(G, 60 * 10**9, np.int64)
    hard = np.full(G, 4000 * 10**9, np.int64)
    one = esc.Context(groups)
    P, N = one.pack(pods, nodes, trackers)
    one.load(P, N)
    one.load_placement(pn, ts, nd)
    want = one.try_remove(now_ns, soft, hard)
    world = 3
    ctxs = []
    for r in range(world):
        lo, hi = shard_range(len(pods), r, world)
        c = esc.Context(groups, rank=r, world=world)
        Pr, Nr = c.pack(pods[lo:hi], nodes, trackers)
        c.load(Pr, Nr, pod_offset=lo)
        c.load_placement(pn[lo:hi], ts, nd)
        c.reap_occupancy()
        ctxs.append(c)
    total = sum(c.reap_download().astype(np.int64) for c in ctxs).astype(np.uint32)
    for c in ctxs:
        c.reap_upload(total)
        got = c.reap_finish(now_ns, soft, hard)
        assert got.tobytes() == want.tobytes()
        for g in range(G):
            assert list(c.removal_nodes(g)) == list(one.removal_nodes(g))
    _check_reaping(one, groups, pods, nodes, trackers, now_ns, soft, hard)


# ------------------------------------------------ dry-mode taintTracker (§8f rank 4)
@pytest.mark.parametrize("seed", range(4))
def test_tracker_updates_vs_literal(esc, seed):
    """Dry-mode bookkeeping in place (esc_tracker_update): each round every dry group
    "untaints" its newest tracked members and "taints" its oldest untracked ones, as
    untaintNewestN / taintOldestN do in dry mode (scale_up.go:146-158,
    scale_down.go:197-200); decisions, both orderings and the tracker lists then equal the
    literal oracle over the updated name slices.  Wet groups' trackers are ignored."""
    rng = random.Random(9700 + seed)
    G = rng.choice([3, 8])
    groups = make_groups(rng, G, with_default=True)
    for g in rng.sample(range(G), max(1, G // 2)):
        groups[g]["dry_mode"] = True
    pods = make_pods(rng, 400, groups, big_frac=0.0)
    nodes = make_nodes(rng, 80, groups, big_frac=0.0)
    states = make_states(rng, G)
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    idx = {nd["name"]: i for i, nd in enumerate(nodes)}
    names = {g: list(trackers.get(g, [])) for g in range(G)}
    ctx.use_graph(True)
    for rnd in range(4):
        tot, dec = ctx.decide_all(states)
        ctx.sort_nodes()
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], pods, nodes, tracker=names[g])
            t, d = tot[g], dec[g]
            assert (t["n_untainted"], t["n_tainted"], t["n_cordoned"]) == \
                (L["n_untainted"], L["n_tainted"], L["n_cordoned"]), (rnd, g)
            assert (t["node_cpu_m"], t["node_mem_b"]) == (L["node_cpu_m"], L["node_mem_b"]), (rnd, g)
            assert int(d["delta"]) == L["delta"] and _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]), (rnd, g)
            unt, tnt = L["untainted"], L["tainted"]
            assert list(ctx.group_order(g, 0)) == [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
            assert list(ctx.group_order(g, 1)) == [tnt[i] for i in O.newest_first([nodes[i]["created_ns"] for i in tnt])]
            assert list(ctx.tracker_list(g)) == sorted({idx[n] for n in names[g] if n in idx}), (rnd, g)
        changes = []                                 # from this round's orderings
        for g in range(G):
            if groups[g].get("dry_mode"):
                rm = list(ctx.group_order(g, 1))[:rng.randrange(0, 4)]
                ad = list(ctx.group_order(g, 0))[:rng.randrange(0, 5)]
            else:                                    # a wet group's tracker changes nothing
                rm = rng.sample(range(len(nodes)), 2)
                ad = [j for j in rng.sample(range(len(nodes)), 3) if nodes[j]["name"] not in names[g]]
            changes.append((rm, ad))
        for g, (rm, ad) in enumerate(changes):
            ctx.tracker_update(g, add=ad, remove=rm)
            for j in rm:                             # untaintNewestN: delete the first equal name
                if nodes[j]["name"] in names[g]:
                    names[g].remove(nodes[j]["name"])
            names[g] += [nodes[j]["name"] for j in ad]
        # node events keep the context's tracker bit whatever the caller packed
        nid = rng.sample(range(len(nodes)), 6)
        for j in nid:
            nodes[j]["taints"] = ["atlassian.com/escalator"] if rng.random() < 0.5 else []
        _, Nn = ctx.pack([], nodes)
        ctx.nodes_update(nid, Nn["flags"][nid], Nn["cpu"][nid], Nn["mem"][nid])
    # refused whole: re-adding a tracked node; removing an untracked one is a no-op
    g = next((g for g in range(G) if ctx.tracker_list(g).size), None)
    if g is not None:
        before = list(ctx.tracker_list(g))
        free = [j for j in range(len(nodes)) if j not in before]
        with pytest.raises(RuntimeError):
            ctx.tracker_update(g, add=free[:1] + before[:1])
        assert list(ctx.tracker_list(g)) == before
        ctx.tracker_update(g, remove=free[:3])
        assert list(ctx.tracker_list(g)) == before


# ------------------------------------------------ controller host state across runs
def test_controller_dry_mode_tracker_across_scans(esc):
    """Dry mode over several scans: taintOldestN appends the names it taints to
    the tracker (scale_down.go:197-200), the next scan's filterNodes counts them as tainted
    (controller.go:126-138), and a scale-up deletes the newest tracked names first
    (untaintNewestN, scale_up.go:146-158).  Every scan equals the literal oracle run with
    the tracker the reference would hold at that point."""
    from escalator_amd.controller import Controller
    opts = {"min_nodes": 5, "max_nodes": 100, "scale_up_pct": 70, "taint_lower_pct": 40, "taint_upper_pct": 60,
            "fast_removal_rate": 4, "slow_removal_rate": 2, "dry_mode": True}
    grp = _default_group(opts)
    nodes = [dict(n, created_ns=1_000_000 + 7919 * ((i * 37) % 10)) for i, n in
             enumerate(build_test_nodes(10, {"CPU": 2000, "Mem": 8000}))]
    ctl = Controller([grp])
    tracker = []                                    # the reference's nodeGroup.taintTracker
    pods = []
    expect_deltas = []
    for scan in range(5):
        if scan == 3:                               # load arrives: scale up, untaint newest
            pods = build_test_pods(60, {"CPU": [500], "Mem": [1000]})
        L = O.scale_node_group(grp, {}, pods, nodes, tracker=list(tracker))
        r = ctl.run_once(lambda: pods, lambda: nodes)[0]
        assert (r["totals"]["n_untainted"], r["totals"]["n_tainted"]) == (L["n_untainted"], L["n_tainted"]), scan
        assert (r["branch"], r["delta"]) == (L["branch"], L["delta"]), (scan, r, L)
        expect_deltas.append(L["delta"])
        # the reference's actuation on its own lists
        if L["delta"] < 0 and L["taint_err"] is None:
            unt = L["untainted"]
            picked = [unt[i] for i in O.taint_oldest_n([nodes[i]["created_ns"] for i in unt], L["n_to_taint"])]
            tracker += [nodes[i]["name"] for i in picked]
            assert r["tainted_now"] == picked, scan
        elif L["delta"] > 0:
            tn = L["tainted"]
            picked = [tn[i] for i in O.newest_first([nodes[i]["created_ns"] for i in tn])][:L["delta"]]
            for i in picked:
                tracker.remove(nodes[i]["name"])
            assert r["untainted_now"] == picked, scan
        assert ctl.taint_tracker[0] == tracker, scan
    assert expect_deltas[:3] == [-4, -4, -4] and expect_deltas[3] > 0


def test_controller_scale_up_cool_down_lock(esc):
    """ScaleUp locks the group with the nodes it added (scale_up.go:39); inside
    ScaleUpCoolDownPeriod every run returns requestedNodes (controller.go:317-323,
    scale_lock.go:22-29), afterwards the lock opens and the delta is computed again."""
    from escalator_amd.controller import Controller
    grp = _default_group({"min_nodes": 0, "max_nodes": 100, "scale_up_pct": 70, "taint_lower_pct": 40,
                          "taint_upper_pct": 60, "fast_removal_rate": 4, "slow_removal_rate": 2,
                          "scale_up_cool_down_ns": 60 * 10**9})
    nodes = build_test_nodes(10, {"CPU": 2000, "Mem": 8000})
    pods = build_test_pods(60, {"CPU": [500], "Mem": [1000]})
    now = [1_700_000_000 * 10**9]
    ctl = Controller([grp], clock=lambda: now[0])
    r = ctl.run_once(lambda: pods, lambda: nodes)[0]
    assert r["branch"] == "scale_up" and r["delta"] == 12 and r["added"] == 12
    now[0] += 30 * 10**9                            # inside the cool-down: locked
    r = ctl.run_once(lambda: pods, lambda: nodes)[0]
    assert (r["branch"], r["delta"]) == ("locked", 12)
    now[0] += 31 * 10**9                            # cool-down over: computed again
    r = ctl.run_once(lambda: pods, lambda: nodes)[0]
    assert (r["branch"], r["delta"]) == ("scale_up", 12)


# ------------------------------------------------ filter truth tables through the HIP path
def test_filter_truth_tables_through_hip(esc, golden):
    """node_group_test.go:13-318 (NewPodAffinityFilterFunc, NewPodDefaultFilterFunc,
    NewNodeLabelFilterFunc truth tables) through pack -> K1 / K2 -> per-group counts: a
    one-group context holding only the case's pod (node) counts it iff the filter selects
    it."""
    fx = golden["controller"]
    for c in fx["pod_affinity_filter"]["cases"]:
        pod = build_test_pod(fx["pod_affinity_filter"]["pods"][c["pod"]])
        ctx = esc.Context([{"name": "g", "label_key": c["key"], "label_value": c["value"], "max_nodes": 10}])
        ctx.load(*ctx.pack([pod], []))
        tot, _ = ctx.decide_all()
        assert int(tot["n_pods"][0]) == int(c["want"]), c["name"]
    for c in fx["pod_default_filter"]["cases"]:
        pod = build_test_pod(fx["pod_default_filter"]["pods"][c["pod"]])
        ctx = esc.Context([{"name": "default", "label_key": "k", "label_value": "v", "max_nodes": 10}])
        ctx.load(*ctx.pack([pod], []))
        tot, _ = ctx.decide_all()
        assert int(tot["n_pods"][0]) == int(c["want"]), c["name"]
    for c in fx["node_label_filter"]["cases"]:
        node = build_test_node(fx["node_label_filter"]["nodes"][c["node"]])
        ctx = esc.Context([{"name": "g", "label_key": c["key"], "label_value": c["value"], "max_nodes": 10}])
        ctx.load(*ctx.pack([], [node]))
        tot, _ = ctx.decide_all()
        assert int(tot["n_nodes"][0]) == int(c["want"]), c["name"]
        ctx.sort_nodes()
        assert len(ctx.group_order(0, 0)) + len(ctx.group_order(0, 1)) + int(tot["n_cordoned"][0]) == int(c["want"])


# ------------------------------------------------ BASELINE.json configs at their stated sizes
def test_config3_full_size_vs_c_oracle(esc):
    """BASELINE config #3 at its stated size: 10M pods / 100k nodes / 100 multi-instance-type
    groups with slack (scale-up deltas and float64 percentages bit-exact)."""
    s = esc.Synth(10_000_000, 100_000, 100, config=3, seed=0xE5CA1A7E00000003, threads=16)
    pods, nodes = s.pods(), s.nodes()
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(True)
    ctx.set_state(s.states)
    for _ in range(3):
        ctx.run()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    assert (dec["branch"] == 7).sum() >= 50, "config 3 is tuned so that most groups scale up"


def test_config2_full_size_vs_c_oracle(esc):
    """BASELINE config #2 (configs[1]) at its stated size: 1M pods / 10k nodes / 100 groups;
    every group's totals and decision, its two orderings and its delivered selection (the
    walk's first need + slack nodes) against the C oracle, through the graph and eagerly."""
    s = esc.Synth(1_000_000, 10_000, 100, config=2, seed=0xE5CA1A7E00000002, threads=16)
    pods, nodes = s.pods(), s.nodes()
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    want = soa.order_all(nodes, s.groups)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(3, 64)
    for graph in (True, False):
        ctx.use_graph(graph)
        for _ in range(2):
            ctx.run()
            tot, dec = ctx.results()
            check_against_c_oracle(tot, dec, otot, odf, odi)
            which, off, idx = ctx.selections()
            for g in range(len(s.groups)):
                for w in (0, 1):
                    assert np.array_equal(ctx.group_order(g, w), want[(g, w)]), (g, w)
                delta, ntt = int(dec["delta"][g]), int(dec["n_to_taint"][g])
                if delta > 0:
                    k, need = 1, delta
                elif delta < 0 and int(dec["taint_status"][g]) == 0:
                    k, need = 0, ntt
                else:
                    assert which[g] == -1, g
                    continue
                c = min(max(need, 0) + 3, len(want[(g, k)]), 64)
                assert which[g] & 3 == k, g
                if which[g] & 4 and off[g + 1] == off[g] and c:   # a tie run too long for the kernel
                    continue
                assert np.array_equal(idx[off[g]:off[g + 1]], want[(g, k)][:c]), g


def test_config4_full_size_vs_c_oracle(esc):
    """BASELINE config #4 at its stated size on one GPU: 100M pods / 1M nodes / 10k groups;
    every group's totals and decision, and every group's two orderings (taintOldestN,
    untaintNewestN), equal the C oracle (the check bench.py makes, here in the GPU suite)."""
    s = esc.Synth(100_000_000, 1_000_000, 10_000, config=4, seed=0xE5CA1A7E00000004, threads=16)
    pods, nodes = s.pods(), s.nodes()
    otot = soa.totals(pods, nodes, s.groups, threads=16)
    odf, odi = soa.decide(s.groups, s.states, otot)
    want = soa.order_all(nodes, s.groups)
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    for _ in range(2):
        ctx.run()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    n = 0
    for g in range(10_000):
        for w in (0, 1):
            got = ctx.group_order(g, w)
            assert np.array_equal(got, want[(g, w)]), (g, w, len(got), len(want[(g, w)]))
            n += len(got)
    assert n > 900_000


def test_config5_full_size_orderings_vs_c_oracle(esc):
    """BASELINE config #5 at its stated size: 10M nodes in 100 groups; every group's
    taint order (untainted oldest first) and untaint order (tainted newest first) equal the
    C oracle's, and the decision's totals too."""
    s = esc.Synth(100_000, 10_000_000, 100, config=5, seed=0xE5CA1A7E00000005, threads=16)
    pods, nodes = s.pods(), s.nodes()
    want = soa.order_all(nodes, s.groups)
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    ctx.run()
    tot, dec = ctx.results()
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    check_against_c_oracle(tot, dec, otot, odf, odi)
    for _ in range(2):
        ctx.sort_nodes()
    n = 0
    for g in range(100):
        for w in (0, 1):
            got = ctx.group_order(g, w)
            assert np.array_equal(got, want[(g, w)]), (g, w, len(got), len(want[(g, w)]))
            n += len(got)
    assert n > 9_000_000


# ------------------------------------------------ RCCL exchange inside the library (§8e)
@pytest.mark.parametrize("graph", [False, True])
def test_rccl_step_world1_vs_c_oracle(esc, graph):
    """esc_comm_unique_id -> esc_comm_init -> esc_step (K1 + K2 + K3 on the shard, the
    in-place ncclAllReduce(int64, SUM) of the pod words on the context's stream, K4) at
    world 1: the RCCL code path a Go host drives through the C ABI alone."""
    s = esc.Synth(2_000_000, 20_000, 10_000, config=4, seed=0xE5CA1A7E00000004)
    otot = soa.totals(s.pods(), s.nodes(), s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s, rank=0, world=1)
    ctx.load_synth(s, replicas=2)
    ctx.use_graph(graph)
    ctx.set_state(s.states)
    uid = esc.Context.comm_unique_id()
    assert len(uid) == 128
    ctx.comm_init(uid, 0, 1)
    for _ in range(3):
        ctx.step()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    (sb, sc), (mb, mc) = ctx.exchange_buffers()
    assert sc == 5 * 10_000 and mc == 0 and mb is None        # the pod words only
    assert ctx.exchange_slice() == (0, 5 * 10_000)
    assert ctx.comm_size() == 1


def test_decision_beyond_int32_round_trips(esc):
    """The decisions travel to the host as compact 32-B records (delta, n_to_taint as
    int32); a scale-up from zero against a tiny cached capacity gives a delta beyond int32
    (calcScaleUpDelta, util.go:21-31) and must come back exact through the full record."""
    groups = [{"name": "a", "label_key": "k", "label_value": "v", "max_nodes": 100, "scale_up_pct": 70,
               "taint_lower_pct": 40, "taint_upper_pct": 60},
              {"name": "b", "label_key": "k", "label_value": "w", "max_nodes": 100, "scale_up_pct": 70}]
    pods = [{"containers": [{"cpu": 1 << 30, "mem": 1 << 20}], "node_selector": {"k": "v"}} for _ in range(20)]
    pods += [{"containers": [{"cpu": 500, "mem": 1000}], "node_selector": {"k": "w"}} for _ in range(5)]
    states = [{"cached_cpu_m": 1, "cached_mem_b": 1}, {}]
    ctx = esc.Context(groups)
    ctx.load(*ctx.pack(pods, []))
    tot, dec = ctx.decide_all(states)
    for g in range(2):
        L = O.scale_node_group(groups[g], states[g], pods, [])
        assert int(dec["delta"][g]) == L["delta"] and esc._lib.BRANCHES[dec["branch"][g]] == L["branch"], (g, L)
        assert (int(dec["cached_cpu_m"][g]), int(dec["cached_mem_b"][g])) == (L["cached_cpu_m"], L["cached_mem_b"])
    assert int(dec["delta"][0]) > (1 << 31)


def test_bound_exchange_buffer_refused_after_growing_reload(esc):
    """the exchange words follow the owner split, which every esc_load_nodes
    recomputes.  A caller-bound buffer sized for the old split must not be overrun after a
    reload that grows it: esc_reduce returns ESC_E_STATE until a buffer of the new size is
    bound (esc_exchange_buffers still reports it), and then the step runs."""
    import torch
    from escalator_amd._lib import ESC_E_STATE
    from escalator_amd.context import node_soa
    s = esc.Synth(200_000, 20_000, 200, config=4, seed=3)
    ctx = esc.Context(s, rank=0, world=2)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    (_, sc), _ = ctx.exchange_buffers()
    buf = torch.zeros(sc, dtype=torch.int64, device="cuda")
    ctx.bind_exchange(buf.data_ptr(), None)
    ctx.reduce()
    ctx.sync()
    # every node into the first group's pair: rank 0 owns that one heavy pair, rank 1 the
    # rest, so the largest owner's group count (the rows per rank) grows
    nodes = {k: v.copy() for k, v in s.nodes().items()}
    nodes["label0"][:] = soa.group_tables(s.groups)["gpair"][0]
    nodes["flags"] &= ~np.uint32(0xFF00)
    nodes["xl_pair"] = np.zeros(0, np.uint32)
    ns, keep = node_soa(nodes)
    assert ctx.lib.esc_load_nodes(ctx.handle, C.byref(ns), 0, len(nodes["flags"])) == 0
    (_, sc2), _ = ctx.exchange_buffers()
    assert sc2 > sc
    assert ctx.lib.esc_reduce(ctx.handle) == ESC_E_STATE
    buf2 = torch.zeros(sc2, dtype=torch.int64, device="cuda")
    ctx.bind_exchange(buf2.data_ptr(), None)
    ctx.reduce()
    ctx.sync()
    ctx.bind_exchange(None, None)
    del keep
