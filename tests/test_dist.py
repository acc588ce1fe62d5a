"""CPU, world_size 2 / 3 over gloo: the N-GPU exchange — sharded pods, the node side split
by pair ownership, one SUM of the per-group words — reproduces the whole-snapshot totals.

No GPU here, so each rank's words are restated from the C oracle in the library's layout
(the pods' words split lo32 / hi; the node words exact on the group's owner
rank, escalator_amd.layout.owner_ranges, and zero elsewhere); the GPU suite checks the
library's own words against the same layout (tests/test_gpu_multi.py)."""
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


def exchange_words(tot_shard: np.ndarray, tot_all: np.ndarray, groups, nodes, rank: int, world: int) -> np.ndarray:
    """One rank's exchange words (esc_exchange_buffers layout): [G][5] pods (cpu lo, cpu hi,
    mem lo, mem hi, count) from its pod shard, then [G][4] nodes (cpu, mem, unt | taint << 32,
    cord | flags << 32) for the groups whose pairs it owns."""
    from escalator_amd import layout
    from oracle import soa
    t = soa.group_tables(groups)
    G = len(groups)
    pw = np.zeros((G, 5), np.int64)
    for k, col in ((0, 0), (2, 1)):
        v = tot_shard[:, col].astype(object)
        pw[:, k] = [int(x) & 0xFFFFFFFF for x in v]
        pw[:, k + 1] = [int(x) >> 32 for x in v]
    pw[:, 4] = tot_shard[:, 2]
    b = layout.owner_ranges(nodes, len(t["pair_ids"]), world)
    own = (np.asarray(t["gpair"]) >= b[rank]) & (np.asarray(t["gpair"]) < b[rank + 1])
    F = soa.TOT_FIELDS
    nx = np.zeros((G, 4), np.int64)
    nx[:, 0] = tot_all[:, F.index("node_cpu_m")]
    nx[:, 1] = tot_all[:, F.index("node_mem_b")]
    nx[:, 2] = tot_all[:, F.index("n_untainted")] | (tot_all[:, F.index("n_tainted")] << 32)
    nx[:, 3] = tot_all[:, F.index("n_cordoned")]
    nx[~own] = 0
    return np.concatenate([pw.ravel(), nx.ravel()])


def decode_words(W: np.ndarray, G: int) -> np.ndarray:
    """The exchanged words back to (pod cpu, pod mem, pods, node cpu, node mem, unt, taint, cord)."""
    pw = W[:G * 5].reshape(G, 5).astype(object)
    nx = W[G * 5:].reshape(G, 4)
    out = np.zeros((G, 8), np.int64)
    out[:, 0] = [int(a) + (int(b) << 32) for a, b in zip(pw[:, 0], pw[:, 1])]
    out[:, 1] = [int(a) + (int(b) << 32) for a, b in zip(pw[:, 2], pw[:, 3])]
    out[:, 2] = W[:G * 5].reshape(G, 5)[:, 4]
    out[:, 3], out[:, 4] = nx[:, 0], nx[:, 1]
    out[:, 5], out[:, 6], out[:, 7] = nx[:, 2] & 0xFFFFFFFF, nx[:, 2] >> 32, nx[:, 3] & 0xFFFFFFFF
    return out


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
    w = exchange_words(t, t, s.groups, s.nodes(), rank, world)
    S, _ = exchange_host(w, np.zeros(0, np.int64))
    if rank == 0:
        out.put(S)
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
        assert np.array_equal(decode_words(S, 64), want), world


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
