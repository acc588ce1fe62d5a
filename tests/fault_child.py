"""Child process of tests/test_gpu_faults.py: one forced-failure scenario on the MEASUREMENT
library (ESC_LIB_PATH=escalator_amd/libescalator_hip_measure.so, whose esc_debug_* entry
points inject the failures; the product library has none), printing one JSON line of what
it observed.  Run in its own process so the product library of the parent test process and
this one never share a process."""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import escalator_amd as esc  # noqa: E402
from escalator_amd import _lib as L  # noqa: E402
from oracle import soa  # noqa: E402


def exact(ctx, pods, nodes, groups, states):
    """Every group's totals and decision equal the C oracle's."""
    otot = soa.totals(pods, nodes, groups)
    odf, odi = soa.decide(groups, states, otot)
    tot, dec = ctx.results()
    ok = all(np.array_equal(tot[n], otot[:, k]) for k, n in enumerate(soa.TOT_FIELDS[:12]))
    ok &= np.array_equal(dec["cpu_pct"].view(np.uint64), odf[:, 0].view(np.uint64))
    ok &= np.array_equal(dec["delta"], odi[:, 0]) and np.array_equal(dec["n_to_taint"], odi[:, 1])
    return bool(ok)


def orders_exact(ctx, nodes, groups):
    want = soa.order_all(nodes, groups)
    return all(np.array_equal(ctx.group_order(g, w), want[(g, w)]) for g in range(len(groups)) for w in (0, 1))


def group_order_rc(lib, ctx, g):
    n = C.c_int64()
    return lib.esc_group_order(ctx.handle, g, 0, None, 0, C.byref(n))


def mode_order(lib):
    """A split ordering's look-back gives up: esc_sync reports ESC_E_ORDER once, the decision's
    totals and decisions stay exact, esc_group_order refuses that ordering, and the next
    decision orders exactly again (in the step, then through esc_sort_nodes)."""
    s = esc.Synth(200_000, 400_000, 40, config=5, seed=0xE5CA1A7E00000005)
    pods, nodes = s.pods(), s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    out = {}
    L.check(lib.esc_debug_lookback_fail(ctx.handle, 1, 0))
    L.check(lib.esc_run(ctx.handle))
    out["sync_rc"] = lib.esc_sync(ctx.handle)
    out["sync_again_rc"] = lib.esc_sync(ctx.handle)
    out["group_order_rc"] = group_order_rc(lib, ctx, 0)
    out["results_exact"] = exact(ctx, pods, nodes, s.groups, s.states)
    L.check(lib.esc_run(ctx.handle))
    out["next_sync_rc"] = lib.esc_sync(ctx.handle)
    out["next_orders_exact"] = orders_exact(ctx, nodes, s.groups)
    L.check(lib.esc_debug_lookback_fail(ctx.handle, 1, 0))
    L.check(lib.esc_sort_nodes(ctx.handle))
    out["sort_sync_rc"] = lib.esc_sync(ctx.handle)
    L.check(lib.esc_sort_nodes(ctx.handle))
    out["sort_next_rc"] = lib.esc_sync(ctx.handle)
    out["sort_orders_exact"] = orders_exact(ctx, nodes, s.groups)
    return out


def mode_listing(lib):
    """The age index's single-pass listing gives up its look-back: the build fails loudly
    (ESC_E_HIP), nothing is ordered from it, and the next build is exact."""
    s = esc.Synth(100_000, 300_000, 30, config=5, seed=0xE5CA1A7E00000005)
    nodes = s.nodes()
    ctx = esc.Context(s)
    ctx.load_synth(s)
    ctx.set_state(s.states)
    out = {}
    L.check(lib.esc_debug_lookback_fail(ctx.handle, 0, 1))
    out["build_rc"] = lib.esc_build_age_index(ctx.handle)
    out["build_again_rc"] = lib.esc_build_age_index(ctx.handle)
    L.check(lib.esc_sort_nodes(ctx.handle))
    out["sync_rc"] = lib.esc_sync(ctx.handle)
    out["orders_exact"] = orders_exact(ctx, nodes, s.groups)
    return out


def mode_patch(lib):
    """Node informer events whose device writes fail after their host-side writes: the
    context refuses decisions (ESC_E_STATE) until esc_load_nodes, then is exact again
    (esc_nodes_update, esc_nodes_add, esc_nodes_delete, esc_tracker_update)."""
    s = esc.Synth(300_000, 20_000, 60, config=4, seed=0xE5CA1A7E00000004)
    pods, nodes = s.pods(), {k: v.copy() for k, v in s.nodes().items()}
    ctx = esc.Context(s)
    ctx.set_spare(0.5)
    ctx.load(pods, nodes)
    ctx.set_state(s.states)
    out = {}

    def reload_and_check(tag, nd):
        ns, keep = esc.context.node_soa(nd)
        out[tag + "_reload_rc"] = lib.esc_load_nodes(ctx.handle, C.byref(ns), 0, len(nd["flags"]))
        del keep
        out[tag + "_after_rc"] = lib.esc_run(ctx.handle)
        out[tag + "_exact"] = exact(ctx, pods, nd, s.groups, s.states)

    ids = np.arange(5, 200, 7, dtype=np.int64)
    flags = nodes["flags"][ids] ^ np.uint32(L.NF_TAINTED)
    cpu = nodes["cpu"][ids] + 1000
    mem = nodes["mem"][ids]
    L.check(lib.esc_debug_fail_patches(ctx.handle, 1))
    out["update_rc"] = lib.esc_nodes_update(ctx.handle, ids.ctypes.data_as(C.POINTER(C.c_int64)), len(ids),
                                            np.ascontiguousarray(flags).ctypes.data_as(C.POINTER(C.c_uint32)),
                                            np.ascontiguousarray(cpu).ctypes.data_as(C.POINTER(C.c_int64)),
                                            np.ascontiguousarray(mem).ctypes.data_as(C.POINTER(C.c_int64)))
    out["update_refused_rc"] = lib.esc_run(ctx.handle)
    nodes["flags"][ids], nodes["cpu"][ids] = flags, cpu
    reload_and_check("update", nodes)

    add = {k: v[:10].copy() for k, v in nodes.items() if k not in ("xl_pair", "trk_node", "trk_group")}
    add["flags"] = add["flags"] & ~np.uint32(0xFF00 | L.NF_TRACKED)        # no extra labels, untracked
    add["xl_pair"] = np.zeros(0, np.uint32)
    add["trk_node"] = np.zeros(0, np.int32)
    add["trk_group"] = np.zeros(0, np.int32)
    ns, keep = esc.context.node_soa(add)
    got = np.zeros(10, np.int64)
    L.check(lib.esc_debug_fail_patches(ctx.handle, 1))
    out["add_rc"] = lib.esc_nodes_add(ctx.handle, C.byref(ns), got.ctypes.data_as(C.POINTER(C.c_int64)))
    del keep
    out["add_refused_rc"] = lib.esc_run(ctx.handle)
    reload_and_check("add", nodes)

    dels = np.array([3, 4, 50], np.int64)
    L.check(lib.esc_debug_fail_patches(ctx.handle, 1))
    out["delete_rc"] = lib.esc_nodes_delete(ctx.handle, dels.ctypes.data_as(C.POINTER(C.c_int64)), len(dels))
    out["delete_refused_rc"] = lib.esc_run(ctx.handle)
    reload_and_check("delete", nodes)
    return out


if __name__ == "__main__":
    lib = L.load()
    assert hasattr(lib, "esc_debug_lookback_fail"), "not the measurement library: %s" % L.LIB_PATH
    lib.esc_debug_lookback_fail.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
    lib.esc_debug_fail_patches.argtypes = [C.c_void_p, C.c_int32]
    res = {"order": mode_order, "listing": mode_listing, "patch": mode_patch}[sys.argv[1]](lib)
    print(json.dumps(res), flush=True)
