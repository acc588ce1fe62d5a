"""GPU: one process driving several shards (esc_ctx_create_multi), the node side split by
pair ownership, and the controller's actuation walk — all against the oracles.

A one-GPU machine runs several shards on its one device with the peer exchange (a device
listed twice); devices=[0] goes through RCCL (ncclCommInitAll with one rank)."""
import random

import numpy as np
import pytest

from oracle import oracle as O
from oracle import soa
from randobj import make_groups, make_nodes, make_pods, make_reaping_cluster, make_states, make_trackers
from test_gpu import _bits, _fits_k, _packed_subset, check_against_c_oracle, check_metrics

pytestmark = pytest.mark.gpu
soa.build()


@pytest.fixture(scope="module")
def esc():
    import escalator_amd
    return escalator_amd


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_multi_device_context_vs_c_oracle(esc, devices):
    """esc_ctx_create_multi: pods split over the shards, every shard's node side the pairs
    it owns, one esc_step = every shard's step + the SUM of the exchange words + K4; totals,
    decisions, gauges and every group's orderings (answered by the owner shard) bit-exact."""
    P, N, G = 300_000, 30_000, 1000
    s = esc.Synth(P, N, G, config=4, seed=11)
    otot = soa.totals(s.pods(), s.nodes(), s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ctx = esc.Context(s, devices=devices)
    ctx.load_synth(s, replicas=2)
    # ncclCommCount with distinct devices (RCCL); 0 on the peer exchange (no communicator)
    assert ctx.comm_size() == (len(devices) if len(set(devices)) == len(devices) else 0)
    assert ctx.counts() == (P, N)
    ctx.set_state(s.states)
    ctx.set_metrics(True)
    ctx.set_order_in_step(True)
    ctx.k1_calibrate(2)
    for _ in range(3):
        ctx.step()
        tot, dec = ctx.results()
        check_against_c_oracle(tot, dec, otot, odf, odi)
    check_metrics(ctx.metrics(), soa.metrics(otot, odf, odi))
    owners = [ctx.group_owner(g) for g in range(G)]
    assert owners == sorted(owners) and set(owners) <= set(range(len(devices)))
    for g in (0, 1, G // 3, G // 2, G - 1):
        for w in (0, 1):
            assert np.array_equal(ctx.group_order(g, w), soa.order(s.nodes(), s.groups, g, w)), (g, w)
    pb, nb = ctx.stream_bytes()
    from escalator_amd import layout
    k = len(devices)
    cuts = [P * i // k for i in range(k + 1)]
    n_gp = len(soa.group_tables(s.groups)["pair_ids"])
    assert pb == sum(layout.pod_bytes(s.pods(), n_gp, a, b) for a, b in zip(cuts, cuts[1:]))
    assert nb == layout.node_bytes(s.nodes(), n_gp, 0, 1)       # the shards' node shares add up to the index


def test_multi_device_shards_equal_per_process_ranks(esc):
    """The multi-device context's shards are the per-process ranks: the same pod shards,
    owner split and exchange words (summed through the host for the per-process contexts,
    whose owners then decide their own groups)."""
    from escalator_amd.dist import merge_owned, shard_range
    P, N, G = 120_000, 20_000, 300
    full = esc.Synth(P, N, G, config=4, seed=21)
    otot = soa.totals(full.pods(), full.nodes(), full.groups)
    odf, odi = soa.decide(full.groups, full.states, otot)
    world = 3
    words, ctxs = [], []
    for r in range(world):
        lo, hi = shard_range(P, r, world)
        s = esc.Synth(P, N, G, config=4, seed=21, p_lo=lo, p_hi=hi)
        c = esc.Context(s, rank=r, world=world)
        c.load_synth(s, pod_offset=lo)
        c.set_state(full.states)
        c.reduce()
        w, _ = c.exchange_download()
        words.append(w)
        ctxs.append((c, s))
    m = esc.Context(full, devices=[0] * world)
    m.load_synth(full)
    m.set_state(full.states)
    m.step()
    tot, dec = m.results()
    check_against_c_oracle(tot, dec, otot, odf, odi)
    W = np.sum(words, axis=0)
    # the SUM's owner-major pod rows -> every group's pod totals (only the pod words travel)
    rows, cap = ctxs[0][0].exchange_rows(full.nodes(), world)
    assert len(W) == world * cap * 5
    pw = W.reshape(world * cap, 5)[rows.astype(np.int64)]
    assert np.array_equal(pw[:, 0] + (pw[:, 1] << 32), otot[:, soa.TOT_FIELDS.index("pod_cpu_m")])
    assert np.array_equal(pw[:, 4], otot[:, soa.TOT_FIELDS.index("n_pods")])
    parts = []
    for r, (c, _) in enumerate(ctxs):
        off, n = c.exchange_slice()
        assert (off, n) == (r * cap * 5, cap * 5)
        c.exchange_upload(W, np.zeros(0, np.int64))
        c.decide()
        t, d = c.results()
        mine = np.array([m.group_owner(g) == r for g in range(G)])
        assert np.array_equal((t["flags"] & 4) == 0, mine), r           # ESC_TF_NOT_OWNED elsewhere
        assert (d["status"][~mine] == 7).all()                          # ESC_ST_NOT_OWNED
        parts.append((t, d))
    check_against_c_oracle(*merge_owned(parts), otot, odf, odi)


@pytest.mark.parametrize("seed", range(3))
def test_multi_device_events_vs_literal(esc, seed):
    """Informer events on a multi-device context: pod upserts / inserts / deletes routed to
    the shard holding the id (all or nothing across shards), node updates / adds / deletes
    on every shard; decisions and orderings equal the literal oracle on the live objects."""
    from escalator_amd._lib import ESC_E_LIMIT
    rng = random.Random(7700 + seed)
    G = rng.choice([4, 9])
    groups = make_groups(rng, G, with_default=True)
    pods = make_pods(rng, 500, groups, big_frac=0.0)
    nodes = make_nodes(rng, 80, groups, big_frac=0.0)
    states = make_states(rng, G)
    ctx = esc.Context(groups, devices=[0, 0, 0])
    ctx.set_spare(2.0)
    P, N = ctx.pack(pods, nodes)
    ctx.load(P, N)
    live = dict(enumerate(pods))
    alive = set(range(len(nodes)))
    next_id = len(pods)
    for rnd in range(3):
        ev_ids, ev_objs = [], []
        for i in rng.sample(sorted(live), 40):
            ev_ids.append(i)
            ev_objs.append(make_pods(rng, 1, groups, big_frac=0.0)[0])
        for _ in range(20):
            ev_ids.append(next_id)
            ev_objs.append(make_pods(rng, 1, groups, big_frac=0.0)[0])
            next_id += 1
        Pe, _ = ctx.pack(ev_objs, [])
        keep = [k for k in range(len(ev_ids)) if _fits_k(Pe, k)]
        assert ctx.pods_upsert([ev_ids[k] for k in keep], _packed_subset(Pe, keep)) == 0
        for k in keep:
            live[ev_ids[k]] = ev_objs[k]
        dels = rng.sample(sorted(live), 30)
        ctx.pods_delete(dels)
        for i in dels:
            del live[i]
        alive_list = sorted(alive)
        nid = rng.sample(alive_list, 10)
        for j in nid:
            nodes[j]["unschedulable"] = rng.random() < 0.3
            nodes[j]["taints"] = ["atlassian.com/escalator"] if rng.random() < 0.4 else []
            nodes[j]["cpu"] = rng.choice([0, 2000, 16000])
        _, Nn = ctx.pack([], nodes)
        ctx.nodes_update(nid, Nn["flags"][nid], Nn["cpu"][nid], Nn["mem"][nid])
        add = make_nodes(rng, 5, groups, big_frac=0.0)
        for x in add:
            x["name"] = "add-%d-%d-%s" % (seed, rnd, x["name"])
        _, Na = ctx.pack([], add)
        ids = ctx.nodes_add(Na)
        assert list(ids) == list(range(len(nodes), len(nodes) + len(add)))
        alive |= set(int(j) for j in ids)
        nodes += add
        gone = rng.sample(sorted(alive), 3)
        ctx.nodes_delete(gone)
        alive -= set(gone)
        rl = rng.sample(sorted(alive), 6)                 # relabels: group moves on every device
        for j in rl:
            x = make_nodes(rng, 1, groups, big_frac=0.0)[0]
            nodes[j] = dict(x, name=nodes[j]["name"], created_ns=nodes[j]["created_ns"])
        _, Nr = ctx.pack([], [nodes[j] for j in rl])
        ctx.nodes_relabel(rl, Nr)
        idx = sorted(alive)                               # snapshot indices of the live nodes
        cur_nodes = [nodes[j] for j in idx]
        cur = [live[i] for i in sorted(live)]
        tot, dec = ctx.decide_all(states)
        ctx.sort_nodes()
        for g in range(G):
            L = O.scale_node_group(groups[g], states[g], cur, cur_nodes)
            t, d = tot[g], dec[g]
            assert (t["n_pods"], t["n_nodes"], t["n_untainted"], t["n_tainted"], t["n_cordoned"]) == \
                (L["n_pods"], L["n_nodes"], L["n_untainted"], L["n_tainted"], L["n_cordoned"]), (rnd, g)
            assert (t["pod_cpu_m"], t["pod_mem_b"], t["node_cpu_m"], t["node_mem_b"]) == \
                (L["pod_cpu_m"], L["pod_mem_b"], L["node_cpu_m"], L["node_mem_b"]), (rnd, g)
            assert int(d["delta"]) == L["delta"] and _bits(d["cpu_pct"]) == _bits(L["cpu_pct"]), (rnd, g)
            unt = [idx[i] for i in L["untainted"]]
            assert list(ctx.group_order(g, 0)) == [unt[i] for i in O.oldest_first([nodes[i]["created_ns"] for i in unt])]
    many = make_pods(rng, 3000, groups, big_frac=0.0)
    Pm, _ = ctx.pack(many, [])
    keep = [k for k in range(len(many)) if _fits_k(Pm, k)]
    before = ctx.decide_all(states)[0].tobytes()
    assert ctx.pods_upsert([next_id + k for k in range(len(keep))], _packed_subset(Pm, keep)) == ESC_E_LIMIT
    assert ctx.decide_all(states)[0].tobytes() == before


def test_multi_device_reaping_vs_literal(esc):
    """TryRemoveTaintedNodes on a multi-device context: every shard's K6 counts its pods,
    the occupancy words are summed across the shards, K7 gives the literal oracle's
    deletions; pod binds routed to their shards keep it current."""
    from escalator_amd.objects import placement
    from test_gpu import _check_reaping
    rng = random.Random(9500)
    G = 7
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, G, 1200, 90)
    trackers = make_trackers(rng, groups, nodes)
    ctx = esc.Context(groups, devices=[0, 0])
    ctx.set_spare(0.5)
    P, N = ctx.pack(pods, nodes, trackers)
    ctx.load(P, N)
    pn, ts, nd = placement(pods, nodes)
    assert ctx.counts() == (len(pods), len(nodes))
    ctx.load_placement(pn, ts, nd)
    soft = np.full(G, 60 * 10**9, np.int64)
    hard = np.full(G, 4000 * 10**9, np.int64)
    _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, soft, hard)
    index = {n["name"]: j for j, n in enumerate(nodes)}
    mv = rng.sample(range(len(pods)), 40)
    to = [rng.choice(nodes)["name"] for _ in mv]
    ctx.pods_bind(mv, [index[t] for t in to])
    for i, t in zip(mv, to):
        pods[i] = dict(pods[i], node_name=t)
    _check_reaping(ctx, groups, pods, nodes, trackers, now_ns, soft, hard)


# ------------------------------------------------ controller actuation
def _group(**kw):
    g = {"name": "default", "label_key": "", "label_value": "", "min_nodes": 0, "max_nodes": 100,
         "scale_up_pct": 70, "taint_lower_pct": 40, "taint_upper_pct": 60, "fast_removal_rate": 4,
         "slow_removal_rate": 2, "scale_up_cool_down_ns": 60 * 10**9}
    g.update(kw)
    return g


def test_controller_scale_up_clamped_at_max(esc):
    """calculateNodesToAdd (scale_up.go:48-56): at MaxSize the cloud add is refused with
    scaleUpCloudProviderNodeGroup's error and no lock (scale_up.go:66-74); scaleNodeGroup
    still returns the computed delta and no error (controller.go:396), and the next run is
    not locked.  Below the max the add is clamped to MaxSize - TargetSize."""
    from builders import build_test_nodes, build_test_pods
    from escalator_amd.controller import Controller
    nodes = build_test_nodes(10, {"CPU": 2000, "Mem": 8000})
    pods = build_test_pods(60, {"CPU": [500], "Mem": [1000]})
    ctl = Controller([_group(max_nodes=10)], clock=lambda: 10**18)
    r = ctl.run_once(lambda: pods, lambda: nodes)[0]
    assert (r["branch"], r["delta"], r["err"], r["added"]) == ("scale_up", 12, None, 0)
    assert r["action_err"].startswith("refusing to scaleup up beyond the maximum size")
    assert not ctl.state[0]["locked"]
    assert ctl.run_once(lambda: pods, lambda: nodes)[0]["branch"] == "scale_up"
    ctl = Controller([_group(max_nodes=15)], clock=lambda: 10**18)
    r = ctl.run_once(lambda: pods, lambda: nodes)[0]
    assert (r["delta"], r["added"]) == (12, 5) and ctl.state[0]["requested_nodes"] == 5


def test_controller_wet_taint_falls_through_failures(esc):
    """taintOldestN / untaintNewestN walk the whole ordering and skip a node whose API write
    fails until n writes succeed (scale_down.go:179-202, scale_up.go:127-160)."""
    from builders import build_test_nodes
    from escalator_amd.controller import Controller, SimulatedCloud
    nodes = [dict(n, created_ns=1_000_000 + 1000 * ((i * 7) % 10))
             for i, n in enumerate(build_test_nodes(10, {"CPU": 2000, "Mem": 8000}))]

    class Flaky(SimulatedCloud):
        def __init__(self, groups, bad):
            super().__init__(groups)
            self.bad, self.calls = set(bad), []

        def taint(self, g, j):
            self.calls.append(j)
            return j not in self.bad

    oldest = sorted(range(10), key=lambda j: nodes[j]["created_ns"])
    grp = _group(min_nodes=2)
    act = Flaky([grp], bad=oldest[:2])
    ctl = Controller([grp], actuator=act)
    r = ctl.run_once(lambda: [], lambda: nodes)[0]                  # no load: fast scale down by 4
    assert r["branch"] == "fast_down" and r["n_to_taint"] == 4
    assert act.calls == oldest[:6] and r["tainted_now"] == oldest[2:6]


def test_controller_reaps_in_scale_down_and_no_change(esc):
    """TryRemoveTaintedNodes runs before tainting (ScaleDown, scale_down.go:23) and in the
    no-change branch (controller.go:377-383): an empty node tainted past the soft grace is
    handed to the cloud group's DeleteNodes."""
    from builders import build_test_nodes, build_test_pods
    from escalator_amd.controller import Controller, SimulatedCloud
    now = 1_700_000_000
    nodes = build_test_nodes(10, {"CPU": 2000, "Mem": 8000})
    for j in (3, 7):
        nodes[j] = dict(nodes[j], taints=["atlassian.com/escalator"], taint_value=str(now - 3600))

    class Rec(SimulatedCloud):
        deleted = []

        def delete_nodes(self, g, js):
            self.deleted.append(list(js))

    for n_pods, branch in ((0, "fast_down"), (22, "none")):
        grp = _group(min_nodes=1, soft_delete_grace_ns=60 * 10**9, hard_delete_grace_ns=7200 * 10**9)
        act = Rec([grp])
        act.deleted = []
        ctl = Controller([grp], actuator=act, clock=lambda: now * 10**9)
        pods = build_test_pods(n_pods, {"CPU": [500], "Mem": [1000]})
        r = ctl.run_once(lambda: pods, lambda: nodes)[0]
        assert r["branch"] == branch, r
        assert r["removed"] == [3, 7] and act.deleted == [[3, 7]]
