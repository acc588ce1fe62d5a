"""One process per GPU: sharded snapshot + one exchange of the per-group int64 words.

The reference has no parallelism (groups run sequentially,
controller.go:416).  Here every rank holds a contiguous shard of the pod SoA and reduces
its 1/world share of the node index; the per-group words are all-reduced with SUM — over
RCCL/xGMI with the ``nccl`` backend (the words live in a torch tensor bound as the
context's exchange buffer, stream-ordered), or host-staged over ``gloo``.  int64 addition
is associative, so any reduction order gives bit-identical totals; every rank then runs
K4 on the same words.  The first-member words (allNodes[0]) need no exchange in this
build (the context reports min_count 0); a MIN all-reduce runs only if one is asked for.
"""
from __future__ import annotations

import os


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
    """Per-decision exchange of one context's words across the process group."""

    def __init__(self, ctx, device_collective: bool):
        import torch
        import torch.distributed as dist
        self.ctx, self.dist, self.torch = ctx, dist, torch
        self.device_collective = device_collective
        (_, sc), (_, mc) = ctx.exchange_buffers()
        self.min_count = mc
        if device_collective:
            dev = torch.device("cuda", torch.cuda.current_device())
            self.words = torch.zeros(sc, dtype=torch.int64, device=dev)
            self.first = torch.zeros(mc, dtype=torch.int64, device=dev) if mc else None
            ctx.bind_exchange(self.words.data_ptr(), self.first.data_ptr() if mc else None)
            ctx.set_stream(torch.cuda.current_stream().cuda_stream)

    def step(self):
        """K1+K2+K3 on this shard, exchange, K4 (all stream-ordered for RCCL)."""
        self.ctx.reduce()
        if self.device_collective:
            self.dist.all_reduce(self.words, op=self.dist.ReduceOp.SUM)
            if self.min_count:
                self.dist.all_reduce(self.first, op=self.dist.ReduceOp.MIN)
        else:
            s, m = self.ctx.exchange_download()
            ts, tm = self.torch.from_numpy(s), self.torch.from_numpy(m)
            self.dist.all_reduce(ts, op=self.dist.ReduceOp.SUM)
            if self.min_count:
                self.dist.all_reduce(tm, op=self.dist.ReduceOp.MIN)
            self.ctx.exchange_upload(ts.numpy(), tm.numpy())
        self.ctx.decide()


def exchange_host(sum_arr, min_arr):
    """Host-side SUM/MIN all-reduce of numpy int64 arrays (gloo) — used by the CPU tests."""
    import torch
    import torch.distributed as dist
    ts = torch.from_numpy(sum_arr.copy())
    tm = torch.from_numpy(min_arr.copy())
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    dist.all_reduce(tm, op=dist.ReduceOp.MIN)
    return ts.numpy(), tm.numpy()
