"""The reload fallback: a full re-pack and re-load of the config-4
snapshot, what a host does when an event batch does not fit the spare room (ESC_E_LIMIT).

    python scripts/bench_reload.py [--pods 100000000] [--reps 2]

Times, on the GPU box's host threads (ESC_HOST_THREADS / OMP_NUM_THREADS, 16 per GPU):
  pack  — esc_packer_create + esc_packer_add_pods / _add_nodes + the dry-mode trackers
          (esc_packer_set_tracker, node names per dry group) + esc_packer_view over the
          snapshot's object structs (esc_synth_objects: what the cgo shim fills from
          *v1.Pod / *v1.Node; the objects themselves are built before the clock starts);
  load  — esc_load_pods + esc_load_nodes of the packer's arrays into a fresh context (one
          replica: the host layout, the H2D copies, the K5 age index);
then one decision on the reloaded snapshot against the C oracle over the generator's own
arrays (bit-exact: the packer's ids for values no group selects differ from the
generator's, the decisions do not).  Prints one JSON line."""
import argparse
import ctypes as C
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
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import escalator_amd as esc
    from escalator_amd import _lib as L
    from oracle import soa
    P, N, G = args.pods, 1_000_000, 10_000
    t0 = time.perf_counter()
    s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, threads=16)
    po, npods, no, nnodes = s.objects()
    gen_s = time.perf_counter() - t0
    lib = L.load()
    # the dry-mode taintTrackers (controller.go:128-133): node names per dry group, as the
    # controller holds them; set on the packer with the objects
    nd = s.nodes()
    trk = {}
    for j, g in zip(nd["trk_node"].tolist(), nd["trk_group"].tolist()):
        trk.setdefault(g, []).append(b"node-%d" % j)
    trk_c = {g: (C.c_char_p * len(v))(*v) for g, v in trk.items()}
    res = {"pack_s": [], "load_s": []}
    tot = dec = None
    for _ in range(args.reps):
        ctx = esc.Context(s, device=0)
        pk = C.c_void_p()
        t0 = time.perf_counter()
        L.check(lib.esc_packer_create(ctx.handle, C.byref(pk)), "esc_packer_create")
        L.check(lib.esc_packer_add_pods(pk, po, npods), "esc_packer_add_pods")
        L.check(lib.esc_packer_add_nodes(pk, no, nnodes), "esc_packer_add_nodes")
        for g, arr in trk_c.items():
            L.check(lib.esc_packer_set_tracker(pk, g, arr, len(arr)), "esc_packer_set_tracker")
        ps, ns = L.PodSoA(), L.NodeSoA()
        L.check(lib.esc_packer_view(pk, C.byref(ps), C.byref(ns)), "esc_packer_view")
        t1 = time.perf_counter()
        L.check(lib.esc_set_replicas(ctx.handle, 1), "esc_set_replicas")
        L.check(lib.esc_load_pods(ctx.handle, C.byref(ps), 0), "esc_load_pods")
        L.check(lib.esc_load_nodes(ctx.handle, C.byref(ns), 0, ns.n_nodes), "esc_load_nodes")
        t2 = time.perf_counter()
        lib.esc_packer_destroy(pk)
        res["pack_s"].append(t1 - t0)
        res["load_s"].append(t2 - t1)
        ctx.set_state(s.states)
        ctx.run()
        tot, dec = ctx.results()
        ctx.close()
    otot = soa.totals(s.pods(), s.nodes(), s.groups, threads=16)
    odf, odi = soa.decide(s.groups, s.states, otot)
    ok = all(np.array_equal(tot[n], otot[:, k]) for k, n in enumerate(soa.TOT_FIELDS[:12]))
    ok &= np.array_equal(dec["delta"], odi[:, 0]) and np.array_equal(dec["cpu_pct"].view(np.uint64),
                                                                        odf[:, 0].view(np.uint64))
    pack, load = min(res["pack_s"]), min(res["load_s"])
    out = {"metric": "reload fallback: pack + load of the config-4 snapshot from object structs",
           "pods": P, "nodes": N, "node_groups": G, "threads": os.environ.get("ESC_HOST_THREADS") or
           os.environ.get("OMP_NUM_THREADS") or "min(16, hardware)",
           "pack_s": pack, "load_s": load, "reload_s": pack + load,
           "pack_objects_per_s": (npods + nnodes) / pack, "object_build_s_untimed": gen_s,
           "raw_s": res, "parity": "bit-exact vs C oracle (10000 groups)" if ok else "MISMATCH"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
