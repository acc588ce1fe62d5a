"""Incremental snapshot ingestion rate (§8f rank 1): informer-style events applied to the
resident config-4 snapshot instead of a reload.

    python scripts/bench_events.py [--pods 100000000] [--batch 1000000]

Loads the config-4 synthetic snapshot with 5 % spare slots per signature class, then
times (a) batches of in-place pod upserts (the pods' own records re-sent under their ids,
the common "status changed" event), (b) batches of deletes followed by re-inserts of the
same records (slot recycling), (c) node taint / allocatable updates, and (d) one full
decision after the events; the decision is checked bit-exact against the C oracle on the
unchanged snapshot content.  Then (e) node deletions and additions (the same records
re-added as new nodes), after (f) node relabels (two sets of nodes trade records: labels,
creation times, flags, allocatable), checked against the C oracle over the permuted
snapshot.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=100_000_000)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--node-batch", type=int, default=1000)
    args = ap.parse_args()
    import escalator_amd as esc
    from oracle import soa
    P, N, G = args.pods, 1_000_000, 10_000
    s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, threads=16)
    pods, nodes = s.pods(), s.nodes()
    ctx = esc.Context(s)
    ctx.set_spare(0.05)                               # pod classes, node slots / entries / K5 regions
    t0 = time.perf_counter()
    ctx.load_synth(s)
    load_s = time.perf_counter() - t0
    ctx.set_state(s.states)
    f = pods["flags"].astype(np.uint64)
    nxc = ((f >> 8) & 0xFF) + ((f >> 16) & 0xFF) + ((f >> 4) & 1)
    nxp = (f >> 24) & 0x3F
    fits = np.flatnonzero((nxc <= 3) & (nxp <= 3))
    oc = np.concatenate([[0], np.cumsum(nxc)]).astype(np.int64)
    op = np.concatenate([[0], np.cumsum(nxp)]).astype(np.int64)
    rng = np.random.default_rng(5)

    def subset(idx):
        out = {k: pods[k][idx] for k in ("flags", "cpu0", "mem0", "pair0")}
        ci = np.concatenate([np.arange(oc[i], oc[i + 1]) for i in idx]) if len(idx) else np.zeros(0, np.int64)
        pi = np.concatenate([np.arange(op[i], op[i + 1]) for i in idx]) if len(idx) else np.zeros(0, np.int64)
        out["xc_cpu"], out["xc_mem"], out["xp_pair"] = pods["xc_cpu"][ci], pods["xc_mem"][ci], pods["xp_pair"][pi]
        return out

    res = {"upsert_in_place_s": [], "delete_s": [], "reinsert_s": [], "node_update_s": []}
    for _ in range(args.rounds):
        ids = np.sort(rng.choice(fits, size=args.batch, replace=False))
        rec = subset(ids)
        t0 = time.perf_counter()
        assert ctx.pods_upsert(ids, rec) == 0
        res["upsert_in_place_s"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        ctx.pods_delete(ids)
        res["delete_s"].append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        assert ctx.pods_upsert(ids, rec) == 0
        res["reinsert_s"].append(time.perf_counter() - t0)
        nid = np.sort(rng.choice(N, size=min(N, args.batch // 10), replace=False))
        t0 = time.perf_counter()
        ctx.nodes_update(nid, nodes["flags"][nid], nodes["cpu"][nid], nodes["mem"][nid])
        res["node_update_s"].append(time.perf_counter() - t0)
    ctx.run()
    tot, dec = ctx.results()
    otot = soa.totals(pods, nodes, s.groups)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ok = all(np.array_equal(tot[n], otot[:, k]) for k, n in enumerate(soa.TOT_FIELDS[:12]))
    ok &= np.array_equal(dec["delta"], odi[:, 0])
    # node informer Add / Delete (esc_nodes_add / esc_nodes_delete): delete a batch of nodes,
    # then add the same records back as new nodes (next snapshot indices); parity of these
    # rounds is covered by tests/test_gpu.py::test_node_add_delete_vs_literal
    xo = np.concatenate([[0], np.cumsum((nodes["flags"].astype(np.int64) >> 8) & 0xFF)]).astype(np.int64)

    def node_subset(idx):
        out = {k: nodes[k][idx] for k in ("flags", "label0", "cpu", "mem", "created_ns")}
        out["flags"] = out["flags"] & ~np.uint32(4)              # the tracker bit is the context's
        xi = np.concatenate([np.arange(xo[i], xo[i + 1]) for i in idx]) if len(idx) else np.zeros(0, np.int64)
        out["xl_pair"] = nodes["xl_pair"][xi]
        out["trk_node"] = np.zeros(0, np.int32)
        out["trk_group"] = np.zeros(0, np.int32)
        return out

    nb = max(1, args.node_batch)
    live, src = np.arange(N), np.arange(N)            # snapshot index, record it holds
    # node informer Updates that change labels and creation times (esc_nodes_relabel): two
    # disjoint sets of nodes trade their records (labels, creation, flags, allocatable), so
    # every node of the batch moves groups and age; then one decision and three groups'
    # orderings against the C oracle over the permuted snapshot
    res["node_relabel_s"] = []
    for r in range(args.rounds + 1):                  # round 0 warms the host mirrors
        pick = rng.choice(N, size=2 * (nb // 2), replace=False)
        a, b = pick[: nb // 2], pick[nb // 2:]
        ids = np.concatenate([a, b])
        rec = node_subset(np.concatenate([src[b], src[a]]))
        t0 = time.perf_counter()
        ctx.nodes_relabel(ids, rec)
        if r:
            res["node_relabel_s"].append(time.perf_counter() - t0)
        src[a], src[b] = src[b].copy(), src[a].copy()
    ctx.run()
    tot, dec = ctx.results()
    xl_parts = [nodes["xl_pair"][xo[i]:xo[i + 1]] for i in src]
    perm = {"flags": (nodes["flags"][src] & ~np.uint32(4)) | (nodes["flags"] & np.uint32(4)),
            "label0": nodes["label0"][src], "cpu": nodes["cpu"][src], "mem": nodes["mem"][src],
            "created_ns": nodes["created_ns"][src], "xl_pair": np.concatenate(xl_parts).astype(np.uint32),
            "trk_node": nodes["trk_node"], "trk_group": nodes["trk_group"]}
    ptot = soa.totals(pods, perm, s.groups)
    pdf, pdi = soa.decide(s.groups, s.states, ptot)
    ok_rl = all(np.array_equal(tot[n], ptot[:, k]) for k, n in enumerate(soa.TOT_FIELDS[:12]))
    ok_rl &= np.array_equal(dec["delta"], pdi[:, 0]) and np.array_equal(dec["cpu_pct"].view(np.uint64),
                                                                         pdf[:, 0].view(np.uint64))
    ctx.sort_nodes()
    for g in (0, G // 2, G - 1):
        for w in (0, 1):
            ok_rl &= np.array_equal(ctx.group_order(g, w), soa.order(perm, s.groups, g, w))
    res["node_delete_s"], res["node_add_s"] = [], []
    for r in range(args.rounds + 1):                  # round 0 warms the host mirrors
        pick = np.sort(rng.choice(len(live), size=nb, replace=False))
        ids = live[pick]
        rec = node_subset(src[pick])
        t0 = time.perf_counter()
        ctx.nodes_delete(ids)
        t_del = time.perf_counter() - t0
        t0 = time.perf_counter()
        new = ctx.nodes_add(rec)
        t_add = time.perf_counter() - t0
        live = np.concatenate([np.delete(live, pick), new])
        src = np.concatenate([np.delete(src, pick), src[pick]])
        if r:
            res["node_delete_s"].append(t_del)
            res["node_add_s"].append(t_add)
    t0 = time.perf_counter()
    ctx.run()
    ctx.sync()
    decide_after_s = time.perf_counter() - t0
    out = {"metric": "incremental snapshot events applied per second (config 4 resident)",
           "pods": P, "batch": args.batch, "full_load_s": load_s,
           "pod_upserts_per_s": args.batch / float(np.median(res["upsert_in_place_s"])),
           "pod_deletes_per_s": args.batch / float(np.median(res["delete_s"])),
           "pod_reinserts_per_s": args.batch / float(np.median(res["reinsert_s"])),
           "node_updates_per_s": (args.batch // 10) / float(np.median(res["node_update_s"])),
           "node_batch": nb,
           "node_deletes_per_s": nb / float(np.median(res["node_delete_s"])),
           "node_adds_per_s": nb / float(np.median(res["node_add_s"])),
           "node_relabels_per_s": 2 * (nb // 2) / float(np.median(res["node_relabel_s"])),
           "parity_after_relabels": ("bit-exact vs C oracle over the permuted snapshot (10000 groups; orderings of "
                                     "groups 0, %d, %d)" % (G // 2, G - 1)) if ok_rl else "MISMATCH",
           "decision_after_node_events_s": decide_after_s,
           "raw_s": res,
           "parity_after_events": "bit-exact vs C oracle (10000 groups)" if ok else "MISMATCH"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
