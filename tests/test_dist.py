"""CPU, world_size 2 over gloo: sharded pods + the SUM exchange of the pods' per-group
words reproduce the whole-snapshot totals (the exchange the N-GPU decision performs with
ncclAllReduce inside the library); every rank reduces the whole node table itself."""
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


def _worker(rank, world, port, out):
    import torch.distributed as dist
    from escalator_amd.context import Synth
    from escalator_amd.dist import exchange_host
    from oracle import soa
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, N, G = 40_000, 3_000, 64
    lo, hi = shard_range(P, rank, world)
    s = Synth(P, N, G, config=4, seed=5, p_lo=lo, p_hi=hi)
    t = soa.totals(s.pods(), s.nodes(), s.groups)        # this rank's pods, every node
    S, F = exchange_host(np.ascontiguousarray(t[:, 0:3]), np.zeros(0, np.int64))
    nodes_local = np.ascontiguousarray(t[:, 3:12])
    if rank == 0:
        out.put((S, nodes_local))
    dist.destroy_process_group()


def test_two_rank_exchange_equals_whole():
    from escalator_amd.context import Synth
    from oracle import soa
    assert [shard_range(10, r, 3) for r in range(3)] == [(0, 4), (4, 7), (7, 10)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    S, NL = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = Synth(40_000, 3_000, 64, config=4, seed=5)
    t = soa.totals(full.pods(), full.nodes(), full.groups)
    assert np.array_equal(S, t[:, 0:3])                    # pod cpu, mem, count: SUM over ranks
    assert np.array_equal(NL, t[:, 3:12])                  # node words and allNodes[0]: rank-local


class _RangeOrders:
    """Stand-in for a context whose K5 streams nodes [lo, hi): group_order = the oracle's
    order over that range (the GPU path is checked against the same oracle in test_gpu)."""

    def __init__(self, nodes, groups, lo, hi):
        self.nodes, self.groups, self.lo, self.hi, self.G = nodes, groups, lo, hi, len(groups)

    def group_order(self, g, which, cap=None):
        from oracle import soa
        return soa.order(self.nodes, self.groups, g, which, self.lo, self.hi, cap)


def _order_worker(rank, world, port, n, out):
    import torch.distributed as dist
    from escalator_amd.context import Synth
    from escalator_amd.dist import gather_orders
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    N, G = 30_000, 12
    s = Synth(1_000, N, G, config=5, seed=0xE5CA1A7E00000005)
    nlo, nhi = shard_range(N, rank, world)
    ctx = _RangeOrders(s.nodes(), s.groups, nlo, nhi)
    res = {w: gather_orders(ctx, w, n, s.nodes()["created_ns"]) for w in (0, 1)}
    if rank == 0:
        out.put(res)
    dist.destroy_process_group()


def test_sharded_orderings_merge_to_whole():
    """Config #5 on N ranks: every rank orders its node range, the per-group prefixes are
    all-gathered and merged (escalator_amd.dist.gather_orders); the merged taint / untaint
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
