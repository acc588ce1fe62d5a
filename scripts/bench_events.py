"""Incremental snapshot ingestion rate (§8f rank 1): informer-style events applied to the
resident config-4 snapshot instead of a reload.

    python scripts/bench_events.py [--pods 100000000] [--batch 1000000]

Loads the config-4 synthetic snapshot with 5 % spare slots per signature class, then
times (a) batches of in-place pod upserts (the pods' own records re-sent under their ids,
the common "status changed" event), (b) batches of deletes followed by re-inserts of the
same records (slot recycling), (c) node taint / allocatable updates, and (d) one full
decision after the events; the decision is checked bit-exact against the C oracle on the
unchanged snapshot content.  Prints one JSON line."""
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
    args = ap.parse_args()
    import escalator_amd as esc
    from oracle import soa
    P, N, G = args.pods, 1_000_000, 10_000
    s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, threads=16)
    pods, nodes = s.pods(), s.nodes()
    ctx = esc.Context(s)
    ctx.set_spare(0.05)
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
    out = {"metric": "incremental snapshot events applied per second (config 4 resident)",
           "pods": P, "batch": args.batch, "full_load_s": load_s,
           "pod_upserts_per_s": args.batch / float(np.median(res["upsert_in_place_s"])),
           "pod_deletes_per_s": args.batch / float(np.median(res["delete_s"])),
           "pod_reinserts_per_s": args.batch / float(np.median(res["reinsert_s"])),
           "node_updates_per_s": (args.batch // 10) / float(np.median(res["node_update_s"])),
           "raw_s": res,
           "parity_after_events": "bit-exact vs C oracle (10000 groups)" if ok else "MISMATCH"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
