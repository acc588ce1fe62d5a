"""GPU, two processes (world 2 over gloo) on device 0: the N > 1 path with the library's
OWN exchange words.

Each rank is its own process with its own context (esc_ctx_create(rank, world)): it loads
its contiguous pod shard and the whole node table, runs its shard step (K1, the fused tail,
its owned node pairs), hands its words to escalator_amd.dist.Exchange (esc_exchange_download
-> torch.distributed reduce_scatter_tensor SUM into its own slice -> esc_exchange_upload) and runs K4 — the
one-process-per-GPU shape bench.py --gpus N runs, with the collective host-staged because
RCCL cannot put two ranks on one device.  Rank 0's and rank 1's totals, decisions and
gauges, and the ranks' merged orderings (dist.gather_orders), are compared with the C
oracle over the UNSHARDED snapshot; sharded reaping (dist.try_remove: the occupancy words
SUM-exchanged) with the literal oracle over every pod.  (tests/test_dist.py keeps the
oracle-restated words as the CPU shadow of this test.)"""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import soa

pytestmark = pytest.mark.gpu
soa.build()

P, N, G, SEED = 300_000, 30_000, 1000, 11
N_SEL = 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_ranks(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=100) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return got


def _decision_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import escalator_amd as esc
    from escalator_amd.dist import Exchange, gather_orders, gather_results, shard_range
    lo, hi = shard_range(P, rank, world)
    s = esc.Synth(P, N, G, config=4, seed=SEED, p_lo=lo, p_hi=hi)
    ctx = esc.Context(s, device=0, rank=rank, world=world)
    ctx.load_synth(s, pod_offset=lo, replicas=2)
    ctx.set_state(s.states)
    ctx.set_metrics(True)
    ctx.set_order_in_step(True)
    ctx.k1_calibrate(2)
    ex = Exchange(ctx, device_collective=False)
    res, own = [], []
    for _ in range(3):                      # replicas rotate: every step a fresh exchange
        ex.step()
        own.append(ctx.results())           # this rank's own groups
        res.append(gather_results(ctx))     # every group, from the owners
    owners = [ctx.group_owner(g) for g in range(G)]
    merged = {w: gather_orders(ctx, w, N_SEL, s.nodes()["created_ns"]) for w in (0, 1)}
    words, _ = ctx.exchange_download()      # this rank's slice holds the SUM the last decide ran on
    off, n = ctx.exchange_slice()
    out.put((rank, dict(res=res, own=own, metrics=ctx.metrics(), owners=owners, merged=merged,
                        slice=words[off:off + n], pod_bytes=ctx.stream_bytes()[0])))
    dist.barrier()
    dist.destroy_process_group()


def test_two_process_exchange_vs_c_oracle():
    import escalator_amd as esc
    from escalator_amd import layout
    from escalator_amd.dist import shard_range
    from test_gpu import check_against_c_oracle, check_metrics
    full = esc.Synth(P, N, G, config=4, seed=SEED)
    otot = soa.totals(full.pods(), full.nodes(), full.groups)
    odf, odi = soa.decide(full.groups, full.states, otot)
    from escalator_amd.dist import merge_owned_metrics
    got = _run_ranks(_decision_worker, 2)
    n_gp = len(soa.group_tables(full.groups)["pair_ids"])
    owners = got[0]["owners"]
    assert owners == got[1]["owners"] and owners == sorted(owners) and set(owners) == {0, 1}
    mine = {r: np.array(owners) == r for r in (0, 1)}
    for r in (0, 1):
        g = got[r]
        for tot, dec in g["res"]:
            check_against_c_oracle(tot, dec, otot, odf, odi)
        for tot, dec in g["own"]:           # a rank decides only its own groups
            assert np.array_equal((tot["flags"] & 4) == 0, mine[r])
            assert (dec["status"][~mine[r]] == 7).all()
        lo, hi = shard_range(P, r, 2)
        assert g["pod_bytes"] == layout.pod_bytes(full.pods(), n_gp, lo, hi)
        # the owner's slice: the SUM of its groups' pod words, nothing else exchanged
        sl = g["slice"].reshape(-1, 5)[:int(mine[r].sum())]
        F = soa.TOT_FIELDS
        assert np.array_equal(sl[:, 0] + (sl[:, 1] << 32), otot[mine[r], F.index("pod_cpu_m")])
        assert np.array_equal(sl[:, 4], otot[mine[r], F.index("n_pods")])
    check_metrics(merge_owned_metrics([got[0]["metrics"], got[1]["metrics"]], owners), soa.metrics(otot, odf, odi))
    for w in (0, 1):
        for g in range(G):
            want = soa.order(full.nodes(), full.groups, g, w, cap=N_SEL)
            assert np.array_equal(got[0]["merged"][w][g], want), (w, g)
            assert np.array_equal(got[1]["merged"][w][g], want), (w, g)


def _reap_worker(rank, world, port, out, seed):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import escalator_amd as esc
    from escalator_amd.dist import shard_range, try_remove
    from escalator_amd.objects import placement
    from randobj import make_reaping_cluster, make_trackers
    rng = random.Random(seed)
    n_g = 8
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, n_g, 1500, 120)
    trackers = make_trackers(rng, groups, nodes)
    pn, ts, nd = placement(pods, nodes)
    lo, hi = shard_range(len(pods), rank, world)
    c = esc.Context(groups, device=0, rank=rank, world=world)
    Pr, Nr = c.pack(pods[lo:hi], nodes, trackers)
    c.load(Pr, Nr, pod_offset=lo)
    c.load_placement(pn[lo:hi], ts, nd)
    soft = np.full(n_g, 60 * 10**9, np.int64)
    hard = np.full(n_g, 4000 * 10**9, np.int64)
    res = try_remove(c, now_ns, soft, hard, device_collective=False)
    rem = [list(c.removal_nodes(g)) for g in range(n_g)]
    out.put((rank, (res, rem)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("seed", [9400, 9401])
def test_two_process_reaping_vs_literal(seed):
    from oracle import oracle as O
    from randobj import make_reaping_cluster, make_trackers
    got = _run_ranks(_reap_worker, 2, seed)
    rng = random.Random(seed)
    groups, pods, nodes, now_ns = make_reaping_cluster(rng, 8, 1500, 120)
    trackers = make_trackers(rng, groups, nodes)
    for g, grp in enumerate(groups):
        L = O.scale_node_group(grp, {}, pods, nodes, tracker=trackers.get(g, []))
        pods_g = O.filtered_list(pods, O.group_pod_filter(grp))
        all_nodes = [x for x in nodes if O.new_node_label_filter_func(grp.get("label_key", ""),
                                                                      grp.get("label_value", ""))(x)]
        tainted = L["tainted"]
        neg, remaining, ks = O.try_remove_tainted_nodes(grp, [nodes[i] for i in tainted], pods_g, all_nodes, now_ns,
                                                        60 * 10**9, 4000 * 10**9, bool(grp.get("dry_mode")))
        for r in (0, 1):
            res, rem = got[r]
            assert int(res[g]["n_candidates"]) == len(tainted), (r, g)
            assert (-int(res[g]["n_delete"]), int(res[g]["pods_remaining"])) == (neg, remaining), (r, g)
            assert rem[g] == [tainted[k] for k in ks], (r, g)
