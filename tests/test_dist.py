"""CPU, world_size 2 / 3 over gloo: the N-GPU exchange — sharded pods, the node side split
by pair ownership, one SUM reduce-scatter of the pods' per-group words to the groups'
owners — reproduces the whole-snapshot totals.

No GPU here, so each rank's words are restated from the C oracle in the library's layout
(the pods' words split lo32 / hi in owner-major rows,
escalator_amd.layout.exchange_rows; the node words computed whole on the group's owner,
escalator_amd.layout.owner_ranges, and never exchanged); the GPU suite checks the library's
own words against the same layout (tests/test_gpu_multi.py, tests/test_gpu_dist.py)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from escalator_amd.dist import shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def exchange_words(tot_shard: np.ndarray, groups, nodes, world: int) -> tuple[np.ndarray, np.ndarray, int]:
    """One rank's exchange words (esc_exchange_buffers layout): [world * cap][5] pod words
    (cpu lo, cpu hi, mem lo, mem hi, count) from its pod shard, group g in row rows[g]."""
    from escalator_amd import layout
    from oracle import soa
    t = soa.group_tables(groups)
    b = layout.owner_ranges(nodes, len(t["pair_ids"]), world)
    rows, cap = layout.exchange_rows(t["gpair"], b)
    pw = np.zeros((world * cap, 5), np.int64)
    for k, col in ((0, 0), (2, 1)):
        v = tot_shard[:, col].astype(object)
        pw[rows, k] = [int(x) & 0xFFFFFFFF for x in v]
        pw[rows, k + 1] = [int(x) >> 32 for x in v]
    pw[rows, 4] = tot_shard[:, 2]
    return pw.ravel(), rows, cap


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    from escalator_amd import layout
    from escalator_amd.context import Synth
    from oracle import soa
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, N, G = 40_000, 3_000, 64
    lo, hi = shard_range(P, rank, world)
    s = Synth(P, N, G, config=4, seed=5, p_lo=lo, p_hi=hi)
    t = soa.totals(s.pods(), s.nodes(), s.groups)        # this rank's pods, every node
    w, rows, cap = exchange_words(t, s.groups, s.nodes(), world)
    mine = torch.zeros(cap * 5, dtype=torch.int64)
    dist.reduce_scatter_tensor(mine, torch.from_numpy(w))    # what esc_exchange does over RCCL
    sl = mine.numpy().reshape(cap, 5)
    tg = soa.group_tables(s.groups)
    b = layout.owner_ranges(s.nodes(), len(tg["pair_ids"]), world)
    own = [g for g in range(G) if b[rank] <= tg["gpair"][g] < b[rank + 1]]
    F = soa.TOT_FIELDS
    res = {}
    for i, g in enumerate(own):                          # the owner's groups: pod SUMs + its node words
        assert rows[g] == rank * cap + i
        res[g] = [int(sl[i, 0]) + (int(sl[i, 1]) << 32), int(sl[i, 2]) + (int(sl[i, 3]) << 32), int(sl[i, 4])] + \
                 [int(t[g, F.index(k)]) for k in ("node_cpu_m", "node_mem_b", "n_untainted", "n_tainted", "n_cordoned")]
    got = [None] * world
    dist.all_gather_object(got, res)
    if rank == 0:
        merged = {}
        for r in got:
            assert not set(r) & set(merged), "a group decided on two ranks"
            merged.update(r)
        out.put(np.array([merged[g] for g in range(G)], np.int64))
    dist.destroy_process_group()


def test_two_and_three_rank_exchange_equals_whole():
    from escalator_amd.context import Synth
    from oracle import soa
    assert [shard_range(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    full = Synth(40_000, 3_000, 64, config=4, seed=5)
    t = soa.totals(full.pods(), full.nodes(), full.groups)
    F = soa.TOT_FIELDS
    want = t[:, [F.index(k) for k in ("pod_cpu_m", "pod_mem_b", "n_pods", "node_cpu_m", "node_mem_b",
                                      "n_untainted", "n_tainted", "n_cordoned")]]
    for world in (2, 3):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        S = q.get(timeout=120)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert np.array_equal(S, want), world


def test_owner_split_library_equals_restatement():
    """The library's owner split (esc_node_owner_ranges, host only) == layout.owner_ranges,
    and it covers every pair exactly once, in rank order."""
    from escalator_amd import layout
    from escalator_amd.context import Context, Synth
    from oracle import soa
    for cfg, P, N, G in ((4, 1000, 30_000, 2000), (5, 1000, 100_000, 100), (2, 1000, 5_000, 7)):
        s = Synth(P, N, G, config=cfg, seed=cfg)
        ctx = Context(s.groups, device=-1)
        n_gp = len(soa.group_tables(s.groups)["pair_ids"])
        for world in (1, 2, 3, 8, 16):
            b = [int(x) for x in ctx.owner_ranges(s.nodes(), world)]
            assert b == layout.owner_ranges(s.nodes(), n_gp, world), (cfg, world)
            assert b[0] == 0 and b[-1] == n_gp and b == sorted(b)
            # owner-major exchange rows: the library's == the restatement's, a permutation
            # into world x cap rows whose block r holds exactly rank r's groups
            rows, cap = ctx.exchange_rows(s.nodes(), world)
            want, wcap = layout.exchange_rows(soa.group_tables(s.groups)["gpair"], b)
            assert cap == wcap and np.array_equal(rows, want), (cfg, world)
            assert len(set(rows.tolist())) == G and int(rows.max()) < world * cap
            gp = soa.group_tables(s.groups)["gpair"]
            assert all(b[r // cap] <= gp[g] < b[r // cap + 1] for g, r in enumerate(rows.tolist()))
        # ranks' node bytes add up to the whole index's
        assert sum(layout.node_bytes(s.nodes(), n_gp, r, 8) for r in range(8)) == layout.node_bytes(s.nodes(), n_gp)


class _OwnerOrders:
    """Stand-in for a context on rank r: K5 orders the groups whose pairs the rank owns
    (layout.owner_ranges), group_order of another rank's group has no members — the oracle's
    order (the GPU path is checked against the same oracle in test_gpu)."""

    def __init__(self, nodes, groups, rank, world):
        from escalator_amd import layout
        from oracle import soa
        t = soa.group_tables(groups)
        b = layout.owner_ranges(nodes, len(t["pair_ids"]), world)
        self.own = [b[rank] <= q < b[rank + 1] for q in t["gpair"]]
        self.nodes, self.groups, self.G = nodes, groups, len(groups)

    def group_order(self, g, which, cap=None):
        from oracle import soa
        if not self.own[g]:
            return np.zeros(0, np.int64)
        return soa.order(self.nodes, self.groups, g, which, cap=cap)


def _order_worker(rank, world, port, n, out):
    import torch.distributed as dist
    from escalator_amd.context import Synth
    from escalator_amd.dist import gather_orders
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, G = 30_000, 12
    s = Synth(1_000, N, G, config=5, seed=0xE5CA1A7E00000005)
    ctx = _OwnerOrders(s.nodes(), s.groups, rank, world)
    res = {w: gather_orders(ctx, w, n, s.nodes()["created_ns"]) for w in (0, 1)}
    if rank == 0:
        out.put(res)
    dist.destroy_process_group()


def test_sharded_orderings_merge_to_whole():
    """Config #5 on N ranks: every rank orders the groups it owns, the per-group prefixes
    are all-gathered (escalator_amd.dist.gather_orders); the gathered taint / untaint
    selections equal the whole-snapshot orders."""
    from escalator_amd.context import Synth
    from oracle import soa
    n = 50
    for world in (2, 3):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_order_worker, args=(r, world, port, n, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = q.get(timeout=120)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        full = Synth(1_000, 30_000, 12, config=5, seed=0xE5CA1A7E00000005)
        for w in (0, 1):
            for g in range(12):
                want = soa.order(full.nodes(), full.groups, g, w, cap=n)
                assert np.array_equal(res[w][g], want), (world, w, g)


def test_merge_orders_ties_by_index():
    """Equal creation times keep ascending snapshot index in both directions (the
    single-rank rule), whichever rank holds them."""
    from escalator_amd.dist import merge_orders
    created = np.array([5, 3, 5, 3, 7, 5], np.int64)
    parts = [np.array([1, 0, 2]), np.array([3, 5, 4])]            # each rank's local oldest-first
    assert list(merge_orders(parts, created, 0, 6)) == [1, 3, 0, 2, 5, 4]
    parts = [np.array([0, 2, 1]), np.array([4, 5, 3])]            # local newest-first
    assert list(merge_orders(parts, created, 1, 4)) == [4, 0, 2, 5]
    assert merge_orders([], created, 0, 3).size == 0


class _ReapShard:
    """Stand-in for a pod-sharded context's reaping steps (esc_reap_occupancy / _download /
    _upload / _finish): occupancy words = this rank's group pods per (group, node), the
    literal oracle's filters; finish = TryRemoveTaintedNodes over the summed words.  The
    GPU path is checked against the same oracle in tests/test_gpu.py."""

    def __init__(self, groups, pods, nodes, trackers):
        self.groups, self.pods, self.nodes, self.trackers = groups, pods, nodes, trackers
        self.G, self.N = len(groups), len(nodes)
        self.index = {n["name"]: j for j, n in enumerate(nodes)}

    def reap_occupancy(self):
        from oracle import oracle as O
        w = np.zeros((self.G, self.N), np.uint32)
        for g, grp in enumerate(self.groups):
            for p in O.filtered_list(self.pods, O.group_pod_filter(grp)):
                j = self.index.get(p.get("node_name") or "")
                if j is not None and not O.pod_is_daemonset(p):
                    w[g, j] += 1
        self.words = w.ravel()

    def reap_download(self):
        return self.words.copy()

    def reap_upload(self, w):
        self.words = np.asarray(w, np.uint32)

    def reap_finish(self, now_ns, soft, hard):
        from oracle import oracle as O
        occ = self.words.reshape(self.G, self.N)
        out = []
        for g, grp in enumerate(self.groups):
            L = O.scale_node_group(grp, {}, [], self.nodes, tracker=self.trackers.get(g, []))
            dels, remaining = [], 0
            for j in L["tainted"]:
                node = self.nodes[j]
                if (node.get("annotations") or {}).get("atlassian.com/no-delete", ""):
                    continue
                t = O.get_to_be_removed_time(node)
                if t is None:
                    continue
                age = now_ns - t * 1_000_000_000
                if age > soft[g] and (occ[g, j] == 0 or age > hard[g]) and not grp.get("dry_mode"):
                    dels.append(j)
                    remaining += int(occ[g, j])
            out.append((len(L["tainted"]), len(dels), remaining))
        return np.array(out, np.int64)


def _reap_worker(rank, world, port, out):
    import random
    import torch.distributed as dist
    from escalator_amd.dist import try_remove
    from randobj import make_reaping_cluster, make_trackers
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = random.Random(77)
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, 6, 500, 60)
    trackers = make_trackers(rng, groups, nodes)
    lo, hi = shard_range(len(pods), rank, world)
    ctx = _ReapShard(groups, pods[lo:hi], nodes, trackers)
    soft = np.full(6, 60 * 10**9, np.int64)
    hard = np.full(6, 3000 * 10**9, np.int64)
    res = try_remove(ctx, now_ns, soft, hard, device_collective=False)
    out.put((rank, res))
    dist.destroy_process_group()


def test_two_rank_sharded_reaping_equals_whole():
    """Sharded TryRemoveTaintedNodes (escalator_amd.dist.try_remove, host-staged over gloo):
    every rank's result equals the literal oracle over the whole pod list."""
    import random
    from oracle import oracle as O
    from randobj import make_reaping_cluster, make_trackers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = random.Random(77)
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, 6, 500, 60)
    trackers = make_trackers(rng, groups, nodes)
    for g, grp in enumerate(groups):
        L = O.scale_node_group(grp, {}, pods, nodes, tracker=trackers.get(g, []))
        pods_g = O.filtered_list(pods, O.group_pod_filter(grp))
        all_nodes = [n for n in nodes if O.new_node_label_filter_func(grp.get("label_key", ""),
                                                                     grp.get("label_value", ""))(n)]
        neg, remaining, _ = O.try_remove_tainted_nodes(grp, [nodes[i] for i in L["tainted"]], pods_g, all_nodes,
                                                       now_ns, 60 * 10**9, 3000 * 10**9, bool(grp.get("dry_mode")))
        for r in (0, 1):
            assert tuple(int(x) for x in got[r][g]) == (len(L["tainted"]), -neg, remaining), (r, g)
