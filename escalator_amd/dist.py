"""One process per GPU: sharded pods, the node side split by pair ownership, and one SUM
reduce-scatter of the pods' per-group words to each group's owner.

The reference has no parallelism (groups run sequentially,
controller.go:416).  Here every rank holds a contiguous shard of the pod SoA and the whole
node table; it reduces, orders and DECIDES the groups whose node pairs it owns (a
contiguous pair range balanced by node entries, the same split on every rank, DESIGN.md
§7).  The pods' per-group words (sums split lo32 / hi, so a cross-rank SUM cannot wrap)
sit in owner-major rows and are reduce-scattered with SUM — by the library's own RCCL
communicator (esc_comm_init / esc_exchange: ncclReduceScatter over xGMI on the context's
stream), or host-staged over ``gloo`` — so every owner receives the exact sums of its own
groups and nothing else; the node words never travel.  int64 addition is associative, so
any reduction order gives bit-identical totals.  A rank's esc_results holds its own groups
(the others flagged ESC_TF_NOT_OWNED); ``gather_results`` collects every group's records
where one host needs them all.  (One process driving every GPU is
``Context(..., devices=[...])``: the same sharding with the exchange inside the library and
the owners' records merged into one result.)
"""
from __future__ import annotations

import os

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced shard [lo, hi) of n records for `rank` (rank order = index order,
    which keeps "first member" = lowest global index = lowest rank with a member)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def env_rank() -> tuple[int, int, int]:
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


class Exchange:
    """Per-decision exchange of one context's pod words across the process group.

    device_collective: the library's own RCCL communicator (esc_comm_init; rank 0's
    unique id travels over the torch.distributed group), one in-place
    ncclReduceScatter(int64, SUM) of the owner-major pod words on the context's stream
    between the shard step and K4 (esc_step) — the path a Go host drives through the C ABI
    alone.  Otherwise host-staged over the group (gloo): download, reduce_scatter into this
    rank's slice, upload."""

    def __init__(self, ctx, device_collective: bool):
        import torch
        import torch.distributed as dist
        self.ctx, self.dist, self.torch = ctx, dist, torch
        self.device_collective = device_collective
        (_, sc), (_, mc) = ctx.exchange_buffers()
        assert mc == 0, "allNodes[0] comes from the whole node table on every rank: nothing to MIN-exchange"
        if device_collective:
            rank, world = dist.get_rank(), dist.get_world_size()
            obj = [ctx.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.comm_init(obj[0], rank, world)

    def step(self):
        """K1+K2+K3 on this shard, exchange, K4."""
        if self.device_collective:
            self.ctx.step()
            return
        self.ctx.reduce()
        s, _ = self.ctx.exchange_download()
        off, n = self.ctx.exchange_slice()
        mine = self.torch.zeros(n, dtype=self.torch.int64)
        self.dist.reduce_scatter_tensor(mine, self.torch.from_numpy(s), op=self.dist.ReduceOp.SUM)
        s[off:off + n] = mine.numpy()
        self.ctx.exchange_upload(s, np.zeros(0, np.int64))
        self.ctx.decide()


def merge_owned(parts):
    """Every group's (totals, decision) from the ranks' esc_results: each group's records
    from the rank that owns it (the others carry ESC_TF_NOT_OWNED in their totals' flags)."""
    from ._lib import ESC_TF_NOT_OWNED
    tot, dec = parts[0][0].copy(), parts[0][1].copy()
    for t, d in parts[1:]:
        m = (t["flags"] & ESC_TF_NOT_OWNED) == 0
        tot[m] = t[m]
        dec[m] = d[m]
    assert not ((tot["flags"] & ESC_TF_NOT_OWNED) != 0).any(), "a group without an owner"
    return tot, dec


def merge_owned_metrics(parts, owners):
    """Every group's gauges (esc_metrics_results) from the rank that owns it."""
    out = parts[0].copy()
    for r, m in enumerate(parts):
        sel = np.asarray(owners) == r
        out[sel] = m[sel]
    return out


def gather_results(ctx):
    """All ranks: every group's totals and decision (the owners' records all-gathered over
    the process group: G x 168 B per rank, outside any timed step)."""
    import torch.distributed as dist
    mine = ctx.results()
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, mine)
    return merge_owned(got)


def try_remove(ctx, now_ns: int, soft_ns, hard_ns, device_collective: bool):
    """TryRemoveTaintedNodes (scale_down.go:51-136) on a pod-sharded context: K6 counts the
    rank's own pods per tainted node, the occupancy words are SUM-all-reduced (uint32) —
    inside the library over RCCL (esc_try_remove) or host-staged over the process group —
    then K7 runs on every rank over the same words, so every rank gets the same deletions."""
    if device_collective:
        return ctx.try_remove(now_ns, soft_ns, hard_ns)
    import torch
    import torch.distributed as dist
    ctx.reap_occupancy()
    w = torch.from_numpy(ctx.reap_download().astype(np.int64))
    dist.all_reduce(w, op=dist.ReduceOp.SUM)
    ctx.reap_upload(w.numpy().astype(np.uint32))
    return ctx.reap_finish(now_ns, soft_ns, hard_ns)


def exchange_host(sum_arr, min_arr):
    """Host-side SUM (and, when non-empty, MIN) all-reduce of numpy int64 arrays (gloo) —
    used by the CPU tests."""
    import torch
    import torch.distributed as dist
    ts = torch.from_numpy(sum_arr.copy())
    tm = torch.from_numpy(min_arr.copy())
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    if tm.numel():
        dist.all_reduce(tm, op=dist.ReduceOp.MIN)
    return ts.numpy(), tm.numpy()


# ------------------------------------------------ sharded orderings (config #5, 1-8 GPUs)
def merge_orders(parts, created_ns, which: int, n: int):
    """Global first `n` of one group's order from the ranks' prefixes.

    The rank owning the group's pair orders all of its members (esc_sort_nodes), the
    others contribute nothing; `which` 0 = untainted oldest-first (taintOldestN,
    scale_down.go:171), 1 = tainted newest-first (untaintNewestN, scale_up.go:118).  The
    merge by creation time with ties by ascending snapshot index — the single-rank tie rule
    — is the general k-way merge, so it also joins prefixes of disjoint node ranges.
    `parts` are int64 arrays of snapshot node indices."""
    import numpy as np
    idx = np.concatenate([np.asarray(p, np.int64) for p in parts]) if parts else np.zeros(0, np.int64)
    if idx.size == 0:
        return idx
    t = np.asarray(created_ns, np.int64)[idx]
    order = np.lexsort((idx, t if which == 0 else -t))   # -t: creation times are far from INT64_MIN
    return idx[order[:n]]


def gather_orders(ctx, which: int, n: int, created_ns, device=None):
    """All ranks: each contributes the first `n` of every group's local order (one
    all_gather of a [G, n + 1] int64 tensor: counts + indices, ≈ G·n·8 B per rank over
    RCCL/xGMI or gloo); returns {group: merged global prefix} (identical on every rank)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    G = ctx.G
    buf = np.full((G, n + 1), -1, np.int64)
    for g in range(G):
        loc = ctx.group_order(g, which, cap=n)[:n]
        buf[g, 0] = len(loc)
        buf[g, 1:1 + len(loc)] = loc
    mine = torch.from_numpy(buf)
    if device is not None:
        mine = mine.to(device)
    world = dist.get_world_size()
    got = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(got, mine)
    got = [x.cpu().numpy() for x in got]
    out = {}
    for g in range(G):
        parts = [x[g, 1:1 + x[g, 0]] for x in got]
        out[g] = merge_orders(parts, created_ns, which, n)
    return out
