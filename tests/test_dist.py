"""CPU, world_size 2 over gloo: sharding + the SUM/MIN exchange reproduce the
whole-snapshot totals (the same exchange the N-GPU bench performs over RCCL)."""
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
    nlo, nhi = shard_range(N, rank, world)
    s = Synth(P, N, G, config=4, seed=5, p_lo=lo, p_hi=hi)
    t = soa.totals(s.pods(), s.nodes(), s.groups, node_lo=nlo, node_hi=nhi)
    first = np.where(t[:, 9] < 0, np.iinfo(np.int64).max, t[:, 9])
    sums = np.delete(t, [9, 10, 11], axis=1)
    S, F = exchange_host(sums, first)
    if rank == 0:
        out.put((S, F))
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
    S, F = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = Synth(40_000, 3_000, 64, config=4, seed=5)
    t = soa.totals(full.pods(), full.nodes(), full.groups)
    want_first = np.where(t[:, 9] < 0, np.iinfo(np.int64).max, t[:, 9])
    sums = np.delete(t, [9, 10, 11], axis=1)
    assert np.array_equal(S[:, :-1], sums[:, :-1])        # flags column: OR semantics, all 0 here
    assert np.array_equal(F, want_first)
