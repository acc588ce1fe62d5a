"""Scale-down reaping (§8f rank 2) at BASELINE config #4: TryRemoveTaintedNodes for all
10k groups over the resident 100M-pod / 1M-node snapshot.

    python scripts/bench_reaping.py [--pods 100000000] [--steps 20] [--warmup 3]

Synthetic bindings (there is no cluster): every pod is bound to a uniformly random node
(2 % to no node), every escalator-tainted node gets a taint time up to 20 minutes old (5 %
unparsable), 1 % of nodes carry the no-delete annotation; soft / hard grace 5 / 15 min.
Times esc_load_placement (once per pod snapshot: the runs, the PodRefs and K6's count of
every entry's occupancy), the node-facts refresh, a batch of pod rescheduling events
(esc_pods_bind: the runs and the occupancy words follow), and esc_try_remove (K7's
per-group pass over the maintained occupancy, including the result download).  Parity: the deletion lists, counts and pods-remaining sums of four
groups against the C oracle (orc_try_remove), which also gives the CPU baseline
(reference-shaped: the group's pods rescanned per group, as TryRemoveTaintedNodes does
through CreateNodeNameToInfoMap; timed on a few groups, extrapolated).  Prints one JSON
line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

NONE = 0xFFFFFFFF
INT64_MIN = np.iinfo(np.int64).min
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    import escalator_amd as esc
    from oracle import soa
    P, N, G = args.pods, 1_000_000, 10_000
    s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, threads=16)
    pods, nodes = s.pods(), s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s)
    rng = np.random.default_rng(11)
    pod_node = rng.integers(0, N, size=P, dtype=np.uint32)
    pod_node[rng.random(P) < 0.02] = NONE
    now_s = 1_800_000_000
    tainted = (nodes["flags"] & 2) != 0
    taint_s = np.where(tainted, now_s - rng.integers(0, 1200, size=N), INT64_MIN).astype(np.int64)
    taint_s[tainted & (rng.random(N) < 0.05)] = INT64_MIN
    no_delete = (rng.random(N) < 0.01).astype(np.uint8)
    now_ns, soft, hard = now_s * 10**9, 300 * 10**9, 900 * 10**9

    ctx.set_spare(0.1)                             # room in every node's run for the bind events
    t0 = time.perf_counter()
    ctx.load_placement(pod_node, taint_s, no_delete)
    place_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx.load_placement(None, taint_s, no_delete)
    refresh_s = time.perf_counter() - t0
    for _ in range(args.warmup):
        ctx.try_remove(now_ns, soft, hard)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = ctx.try_remove(now_ns, soft, hard)
    call_ms = (time.perf_counter() - t0) / args.steps * 1e3
    # the same call through the C ABI with the argument and result arrays made once (what a
    # cgo caller does): the Python wrapper's share of call_ms is the difference
    import ctypes as C
    from escalator_amd import _lib as L
    s_arr = np.full(G, soft, np.int64)
    h_arr = np.full(G, hard, np.int64)
    o_arr = np.empty(G, esc.context.REMOVAL_DTYPE)
    ps, ph = s_arr.ctypes.data_as(C.POINTER(C.c_int64)), h_arr.ctypes.data_as(C.POINTER(C.c_int64))
    po = o_arr.ctypes.data_as(C.POINTER(L.Removal))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        L.check(ctx.lib.esc_try_remove(ctx.handle, int(now_ns), ps, ph, po), "esc_try_remove")
    abi_ms = (time.perf_counter() - t0) / args.steps * 1e3
    assert np.array_equal(o_arr, res)

    # pod rescheduling events (esc_pods_bind) keep the occupancy words current: time a
    # batch, then one call again (its result is the one checked below)
    mv = rng.choice(P, size=100_000, replace=False).astype(np.int64)
    to = rng.integers(0, N, size=len(mv), dtype=np.uint32)
    back = pod_node[mv].copy()
    t0 = time.perf_counter()
    ctx.pods_bind(mv, to)
    bind_s = time.perf_counter() - t0
    pod_node[mv] = to
    ctx.pods_bind(mv, back)                        # and back (both moves are deltas)
    pod_node[mv] = back
    res = ctx.try_remove(now_ns, soft, hard)

    # parity + CPU baseline on four groups
    parity, cpu_s = True, []
    for g in (0, 37, 4242, G - 1):
        t0 = time.perf_counter()
        (cand, ndel, rem), idx = soa.try_remove(pods, nodes, s.groups, pod_node, taint_s, no_delete, g, now_ns,
                                                soft, hard)
        cpu_s.append(time.perf_counter() - t0)
        r = res[g]
        parity &= (int(r["n_candidates"]), int(r["n_delete"]), int(r["pods_remaining"])) == (cand, ndel, rem)
        parity &= np.array_equal(ctx.removal_nodes(g), idx)

    # algorithmic bytes of one call: K6 scans the pair-major entries (flags, pair, node:
    # 12 B) and, per entry of a group pair on a wet-tainted node, the node's run offsets
    # (8 B) and PodRefs (20 B per pod) and writes two counts (8 B); K7 reads each group's
    # entries (flags, node: 8 B) and, per candidate, taint time 8 + no-delete 1 + count 4.
    t = soa.group_tables(s.groups)
    n_gp = t["n_gp"]
    xl_n = (nodes["flags"] >> 8) & 0xFF
    ent_node = np.concatenate([np.flatnonzero(nodes["label0"] != NONE), np.repeat(np.arange(N), xl_n)])
    ent_pair = np.concatenate([nodes["label0"][nodes["label0"] != NONE], nodes["xl_pair"]])
    E = len(ent_node)
    run = np.bincount(pod_node[pod_node != NONE], minlength=N).astype(np.int64)
    wet = ((nodes["flags"] & 2) != 0) & ((nodes["flags"] & 1) == 0)
    proc = (ent_pair < n_gp) & wet[ent_node]
    k6 = 12 * E + int((16 + 20 * run[ent_node[proc]]).sum())
    per_pair = np.bincount(ent_pair[ent_pair < n_gp], minlength=n_gp)
    cand_pair = np.bincount(ent_pair[proc], minlength=n_gp)
    k7 = int(8 * per_pair[t["gpair"]].sum() + 13 * cand_pair[t["gpair"]].sum() + 32 * G)
    cpu_per_group = float(np.median(cpu_s))
    out = {
        "metric": "config4 scale-down reaping: TryRemoveTaintedNodes for every group per call",
        "value": G / (call_ms * 1e-3),
        "unit": "groups/s",
        "ms_per_call": call_ms,
        "ms_per_call_abi": abi_ms,          # the same call with arrays made once (C-ABI caller)
        "steps": args.steps,
        "data": "synthetic (esc_synth.cpp config 4 + random pod bindings / taint times)",
        "config": {"workload": "config4: 100M pods / 1M nodes / 10k groups", "pods": P, "nodes": N,
                   "node_groups": G, "entries": E, "entries_wet_tainted_group_pair": int(proc.sum()),
                   "pods_on_those": int(run[ent_node[proc]].sum())},
        "algorithmic_bytes": {"k_try_remove": k7, "call_GBps": k7 / (call_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                              "k_occupancy_recount": k6,
                              "note": "a call is K7 + the result copy: the per-entry occupancy words are counted "
                                      "once by K6 at esc_load_placement (k_occupancy_recount: its bytes for the "
                                      "wet-tainted entries) and kept current by pod events"},
        "load_placement_s": place_s, "refresh_node_facts_s": refresh_s,
        "pod_binds_per_s": len(mv) / bind_s,
        "deletions": int(res["n_delete"].sum()), "candidates": int(res["n_candidates"].sum()),
        "cpu_baseline": {"value": 1.0 / cpu_per_group, "unit": "groups/s", "cores": 1, "kind": "port",
                         "sample": "oracle/esc_oracle.c orc_try_remove on groups 0, 37, 4242, %d of the same "
                                   "snapshot (one 100M-pod rescan per group, as the reference's per-group "
                                   "CreateNodeNameToInfoMap), median %.2f s/group" % (G - 1, cpu_per_group)},
        "parity": "bit-exact vs C oracle on groups 0, 37, 4242, %d" % (G - 1) if parity else "MISMATCH",
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
