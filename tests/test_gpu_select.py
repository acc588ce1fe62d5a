"""GPU: the taint / untaint selections delivered with the decision (esc_set_selections /
esc_selections) against the C oracle's orderings.

The reference ends a decision in a walk down one ordering (controller.go:367-383):
ScaleDown -> taintOldestN over the untainted nodes oldest first (scale_down.go:171-205),
ScaleUp -> untaintNewestN over the tainted nodes newest first (scale_up.go:118-163), both
skipping a node whose API write fails.  K4 writes every decided group's walk prefix —
need (n_to_taint or delta) + slack nodes, at most group_cap — straight to pinned memory in
the step.  Checked here: every group's list equals the prefix of soa.order (the oracle's
order, ties by ascending snapshot index), the which / cut flags, equal creation times (short
runs resolved in the kernel, runs past SEL_TIE_MAX handed back as a cut), graphs, the
multi-device context, and the Python controller walking them with failing writes."""
import numpy as np
import pytest

from oracle import soa

pytestmark = pytest.mark.gpu
soa.build()

SEL_TIE_MAX = 64
SEL_NONE, SEL_TAINT, SEL_UNTAINT, SEL_CUT = -1, 0, 1, 4


@pytest.fixture(scope="module")
def esc():
    import escalator_amd
    return escalator_amd


def _long_tie(created, order, c):
    """A run of equal creation times longer than SEL_TIE_MAX + 1 touching the first c entries."""
    t = np.asarray(created, np.int64)[np.asarray(order, np.int64)]
    a = 0
    while a < min(c, len(t)):
        b = a
        while b < len(t) and t[b] == t[a]:
            b += 1
        if b - a > SEL_TIE_MAX:
            return True
        a = b
    return False


def check_selections(ctx, dec, want, created, slack, cap, owned=None):
    """Every (owned) group's selection == the oracle walk's prefix; returns the counts of
    (taint lists, untaint lists, cut lists, tie cuts)."""
    which, off, idx = ctx.selections()
    seen = [0, 0, 0, 0]
    for g in range(len(which)):
        if owned is not None and not owned[g]:
            assert which[g] == SEL_NONE, g
            continue
        delta, ntt, ts = int(dec["delta"][g]), int(dec["n_to_taint"][g]), int(dec["taint_status"][g])
        got = idx[off[g]:off[g + 1]]
        if delta > 0:
            w, need = SEL_UNTAINT, delta
        elif delta < 0 and ts == 0:
            w, need = SEL_TAINT, ntt
        else:
            assert which[g] == SEL_NONE and len(got) == 0, (g, which[g], delta)
            continue
        order = want[(g, w)]
        c = min(max(need, 0) + slack, len(order))
        assert which[g] & ~SEL_CUT == w, (g, which[g], w)
        if which[g] & SEL_CUT and len(got) == 0 and c > 0:   # a tie run too long for the kernel
            assert w == SEL_UNTAINT and _long_tie(created, order, min(c, cap)), g
            seen[3] += 1
            continue
        assert bool(which[g] & SEL_CUT) == (c > cap), (g, which[g], c, cap)
        assert np.array_equal(got, order[:min(c, cap)]), (g, w, list(got[:8]), list(order[:8]))
        seen[w] += 1
        seen[2] += c > cap
    return seen


def _snapshot(esc, P, N, G, coarse=0, seed=0xE5CA1A7E00000004):
    s = esc.Synth(P, N, G, config=4, seed=seed, threads=16)
    pods, nodes = s.pods(), s.nodes()
    nodes = {k: v.copy() for k, v in nodes.items()}
    if coarse:                                            # equal creation times (1-s k8s stamps)
        base = int(nodes["created_ns"].min())
        nodes["created_ns"] = base + (nodes["created_ns"] - base) // coarse * coarse
    return s, pods, nodes


@pytest.mark.parametrize("coarse,slack,cap,graph", [(0, 2, 64, False), (0, 0, 3, True),
                                                    (4_000_000, 3, 256, False), (4_000_000, 1, 8, True)])
def test_selections_vs_oracle_orders(esc, coarse, slack, cap, graph):
    """Config-4-shaped snapshot (1 000 groups): every group's selection over several
    decisions, with unique and with coarse (tied) creation times, small group_cap cuts and
    graph replay."""
    s, pods, nodes = _snapshot(esc, 2_000_000, 50_000, 1000, coarse)
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    want = soa.order_all(nodes, s.groups)
    ctx = esc.Context(s)
    ctx.load(pods, nodes, replicas=2)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(slack, cap)
    ctx.use_graph(graph)
    for _ in range(3):
        ctx.run()
        tot, dec = ctx.results()
        assert np.array_equal(dec["delta"], odi[:, 0])
        seen = check_selections(ctx, dec, want, nodes["created_ns"], slack, cap)
    assert seen[SEL_TAINT] >= 50 and seen[SEL_UNTAINT] >= 20, seen
    if cap < 10:
        assert seen[2] > 0, seen                           # some lists were cut at group_cap


def test_selections_long_tie_runs_fall_back(esc):
    """Every node of a group created in the same second: the kernel resolves runs of equal
    times up to SEL_TIE_MAX each way; a longer run comes back as a cut with no nodes, and
    esc_group_order (which reads on until the run ends) gives the walk."""
    s, pods, nodes = _snapshot(esc, 500_000, 40_000, 20, coarse=10**15)   # ~2 000 nodes a group
    want = soa.order_all(nodes, s.groups)
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load(pods, nodes)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(4, 64)
    ctx.run()
    tot, dec = ctx.results()
    seen = check_selections(ctx, dec, want, nodes["created_ns"], 4, 64)
    which, off, idx = ctx.selections()
    for g in np.nonzero((which >= 0) & ((which & SEL_CUT) != 0))[0][:5]:
        w = int(which[g]) & 3
        assert np.array_equal(ctx.group_order(int(g), w), want[(int(g), w)]), g
    long_up = [g for g in range(len(odi)) if odi[g, 0] > 0
               and _long_tie(nodes["created_ns"], want[(g, SEL_UNTAINT)], min(odi[g, 0] + 4, 64))]
    assert seen[SEL_TAINT] > 0 and len(long_up) > 0, (seen, long_up)
    assert seen[3] == len(long_up), (seen, long_up)


def test_selections_config4_full_size(esc):
    """BASELINE config #4 at its stated size (100M pods / 1M nodes / 10k groups): every
    group's selection of every decision against the oracle's orderings."""
    s = esc.Synth(100_000_000, 1_000_000, 10_000, config=4, seed=0xE5CA1A7E00000004, threads=16)
    pods, nodes = s.pods(), s.nodes()
    otot = soa.totals(pods, nodes, s.groups, threads=16)
    odf, odi = soa.decide(s.groups, s.states, otot)
    want = soa.order_all(nodes, s.groups)
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(4, 256)
    for _ in range(2):
        ctx.run()
        tot, dec = ctx.results()
        assert np.array_equal(dec["delta"], odi[:, 0]) and np.array_equal(dec["n_to_taint"], odi[:, 1])
        seen = check_selections(ctx, dec, want, nodes["created_ns"], 4, 256)
    assert seen[SEL_TAINT] + seen[SEL_UNTAINT] > 1000, seen


@pytest.mark.parametrize("devices", [[0], [0, 0, 0]])
def test_selections_multi_device(esc, devices):
    """A multi-device context: every shard delivers its own groups' selections, esc_selections
    merges them by owner."""
    s, pods, nodes = _snapshot(esc, 600_000, 30_000, 500, coarse=2_000_000)
    want = soa.order_all(nodes, s.groups)
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s, devices=devices)
    ctx.load(pods, nodes)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(2, 32)
    for _ in range(2):
        ctx.step()
        tot, dec = ctx.results()
        assert np.array_equal(dec["delta"], odi[:, 0])
        seen = check_selections(ctx, dec, want, nodes["created_ns"], 2, 32)
    assert seen[SEL_TAINT] > 0 and seen[SEL_UNTAINT] > 0, seen


def test_selections_off_and_state(esc):
    """Selections are refused before they are turned on (ESC_E_STATE) and after they are
    turned off; turning them on again delivers the next decision's."""
    from escalator_amd._lib import EscError, ESC_E_STATE
    s, pods, nodes = _snapshot(esc, 200_000, 10_000, 100)
    ctx = esc.Context(s)
    ctx.load(pods, nodes)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.run()
    with pytest.raises(EscError) as e:
        ctx.selections()
    assert e.value.code == ESC_E_STATE
    ctx.set_selections(0, 16)
    ctx.run()
    ctx.results()
    which, off, idx = ctx.selections()
    assert len(off) == 101 and off[-1] == len(idx)
    ctx.set_selections(-1, 0)
    with pytest.raises(EscError):
        ctx.selections()


def test_controller_walks_selections_and_falls_back(esc):
    """The Python controller walks the delivered selections; when failed taint writes use up
    the slack it continues on esc_group_order (the reference's walk goes on down the whole
    order, scale_down.go:179-202)."""
    from builders import build_test_nodes
    from escalator_amd.controller import Controller, SimulatedCloud
    nodes = [dict(n, created_ns=1_000_000 + 1000 * ((i * 7) % 20))
             for i, n in enumerate(build_test_nodes(20, {"CPU": 2000, "Mem": 8000}))]

    class Flaky(SimulatedCloud):
        def __init__(self, groups, bad):
            super().__init__(groups)
            self.bad, self.calls = set(bad), []

        def taint(self, g, j):
            self.calls.append(j)
            return j not in self.bad

    oldest = sorted(range(20), key=lambda j: nodes[j]["created_ns"])
    grp = {"name": "default", "label_key": "", "label_value": "", "min_nodes": 2, "max_nodes": 100,
           "scale_up_pct": 70, "taint_lower_pct": 40, "taint_upper_pct": 60, "fast_removal_rate": 4,
           "slow_removal_rate": 2}
    for slack, bad in ((1, oldest[:1]), (1, oldest[:5]), (0, oldest[:3])):
        act = Flaky([grp], bad=bad)
        ctl = Controller([grp], actuator=act, selection_slack=slack)
        r = ctl.run_once(lambda: [], lambda: nodes)[0]
        assert r["branch"] == "fast_down" and r["n_to_taint"] == 4
        good = [j for j in oldest if j not in set(bad)][:4]
        assert act.calls == oldest[:oldest.index(good[-1]) + 1], (slack, bad)
        assert r["tainted_now"] == good
        assert r["walk_fallback"] == (len(bad) > slack), (slack, bad, r["walk_fallback"])


def _relabel(nodes, groups, sizes, seed=0):
    """The node table with its nodes reassigned so that group g's label pair holds sizes[g]
    nodes (no extra labels, no trackers; the rest unlabelled), in a shuffled order."""
    t = soa.group_tables(groups)
    n = len(nodes["flags"])
    assert sum(sizes) <= n
    lab = np.full(n, 0xFFFFFFFF, np.uint32)
    at = 0
    for g, k in enumerate(sizes):
        lab[at:at + k] = t["gpair"][g]
        at += k
    np.random.default_rng(seed).shuffle(lab)
    out = {k: v.copy() for k, v in nodes.items()}
    out["label0"] = lab
    out["flags"] = out["flags"] & ~np.uint32(0xFF00 | 4)          # no extra labels, not tracked
    out["xl_pair"] = np.zeros(0, np.uint32)
    out["trk_node"] = np.zeros(0, np.int32)
    out["trk_group"] = np.zeros(0, np.int32)
    return out


@pytest.mark.parametrize("shape", ["mixed", "sparse"])
def test_packed_chunk_mix(esc, shape):
    """Region sizes around the chunk limits: small (<= 1024), mid-size (<= 4096, packed up to
    4096) and split groups interleaved — a mid-size chunk followed by a small group was
    dropped (never ordered) before round 6 — and ('sparse') 20 000 groups of which every 50th
    has members, so that packed chunks span more groups than ORD_GCAP.  Every group's two
    orderings and selections against the oracle."""
    rng = np.random.default_rng(5)
    if shape == "mixed":
        G = 200
        pick = rng.integers(0, 5, G)
        sizes = [int(x) for x in np.choose(pick, [rng.integers(0, 60, G), rng.integers(60, 1000, G),
                                                  rng.integers(1025, 4097, G), rng.integers(4097, 9000, G),
                                                  np.zeros(G, np.int64)])]
    else:
        G = 20_000
        sizes = [5 if g % 50 == 0 else 0 for g in range(G)]
    s = esc.Synth(50_000, sum(sizes) + 100, G, config=4, seed=77)
    pods = s.pods()
    nodes = _relabel(s.nodes(), s.groups, sizes)
    want = soa.order_all(nodes, s.groups)
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s)
    ctx.load(pods, nodes)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(1, 64)
    for _ in range(2):
        ctx.run()
        tot, dec = ctx.results()
        assert np.array_equal(dec["delta"], odi[:, 0])
        for g in range(G):
            for w in (0, 1):
                assert np.array_equal(ctx.group_order(g, w), want[(g, w)]), (g, w, sizes[g])
        check_selections(ctx, dec, want, nodes["created_ns"], 1, 64)


def test_selections_ties_from_node_adds(esc):
    """The tie rule is applied per group, only where equal creation times exist
    (RegionSink::tie): a group loaded with unique times copies its tainted segment as is;
    node additions with the creation times of its newest tainted nodes flag it, and its
    untaint list (newest first, equal times by ascending index) still equals the literal
    order; a second group, never given a tie, keeps copying."""
    from builders import build_test_node, build_test_pods
    from oracle import oracle as O
    grp = {"label_key": "k", "min_nodes": 0, "max_nodes": 10_000, "scale_up_pct": 70, "taint_lower_pct": 10,
           "taint_upper_pct": 20, "fast_removal_rate": 4, "slow_removal_rate": 2}
    groups = [dict(grp, name="a", label_value="a"), dict(grp, name="b", label_value="b")]
    nodes = []
    for v in ("a", "b"):
        for i in range(300):                               # unique times; 200 tainted, 100 not
            nodes.append(build_test_node({"Name": "%s%d" % (v, i), "LabelKey": "k", "LabelValue": v,
                                          "CPU": 1000, "Mem": 1 << 30, "Tainted": i % 3 != 0,
                                          "Creation": 10**12 + 7919 * ((i * 37) % 300) + (v == "b")}))
    pods = []
    for v in ("a", "b"):                                   # far over the untainted capacity: ScaleUp
        pods += build_test_pods(400, {"CPU": [900], "Mem": [1 << 20], "NodeSelectorKey": "k",
                                      "NodeSelectorValue": v})
    ctx = esc.Context(groups)
    ctx.set_spare(1.0)
    P, N = ctx.pack(pods, nodes)
    ctx.load(P, N)
    states = [{"locked": False, "requested_nodes": 0, "cached_cpu_m": 0, "cached_mem_b": 0}] * 2
    ctx.set_state(states)
    ctx.set_order_in_step(True)
    ctx.set_selections(2, 64)

    def check(lst, tied):
        ctx.run()
        tot, dec = ctx.results()
        which, off, idx = ctx.selections()
        for g, v in enumerate(("a", "b")):
            assert int(dec["delta"][g]) > 0 and which[g] & 3 == SEL_UNTAINT, (g, dec["delta"][g], which[g])
            tn = [j for j, nd in enumerate(lst) if nd["labels"].get("k") == v and nd["taints"]]
            want = [tn[i] for i in O.newest_first([lst[j]["created_ns"] for j in tn])]
            assert list(ctx.group_order(g, 1)) == want
            c = min(int(dec["delta"][g]) + 2, len(want))
            assert list(idx[off[g]:off[g + 1]]) == want[:min(c, 64)], (g, list(idx[off[g]:off[g] + 6]), want[:6])
            head = [lst[j]["created_ns"] for j in want[:c]]
            assert (len(set(head)) < len(head)) == (tied and v == "a"), g   # the case at hand

    check(nodes, False)
    newest = [j for j in O.newest_first([nd["created_ns"] for nd in nodes[:300]]) if nodes[j]["taints"]][:5]
    add = [build_test_node({"Name": "x%d" % k, "LabelKey": "k", "LabelValue": "a", "CPU": 1000, "Mem": 1 << 30,
                            "Tainted": True, "Creation": nodes[j]["created_ns"]}) for k, j in enumerate(newest[::-1])]
    _, packed = ctx.pack([], add)
    ids = ctx.nodes_add(packed)
    assert list(ids) == list(range(600, 605))
    check(nodes + add, True)
    # group b: a relabel (esc_nodes_relabel) moves one of its tainted nodes' creation time
    # onto its newest tainted node's: b now has equal times in its walk prefix too
    lst = nodes + add
    nb = [j for j in O.newest_first([nd["created_ns"] for nd in nodes[300:]]) if nodes[300 + j]["taints"]]
    newest_b, mover = 300 + nb[0], 300 + nb[10]
    moved = dict(lst[mover], created_ns=lst[newest_b]["created_ns"])
    ctx.nodes_relabel([mover], ctx.pack([], [moved])[1])
    lst = lst[:mover] + [moved] + lst[mover + 1:]
    ctx.run()
    tot, dec = ctx.results()
    which, off, idx = ctx.selections()
    for g, v in enumerate(("a", "b")):
        tn = [j for j, nd in enumerate(lst) if nd["labels"].get("k") == v and nd["taints"]]
        want = [tn[i] for i in O.newest_first([lst[j]["created_ns"] for j in tn])]
        c = min(int(dec["delta"][g]) + 2, len(want), 64)
        assert which[g] & 3 == SEL_UNTAINT and list(idx[off[g]:off[g + 1]]) == want[:c], (g, want[:4])
    assert {newest_b, mover} <= set(idx[off[1]:off[1] + 3].tolist())
