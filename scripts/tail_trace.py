"""The post-K1 chain block by block (measurement library, ESC_TAIL_TRACE=1): for config 4
and rank 0 of 8, every block's start and end in K1 (esc_k1_trace), k_step_tail (by role:
K2 node pieces, tracker, K3 fold, packed orderings) and k_node_groups (esc_debug_tail_trace),
on the one s_memrealtime clock (100 MHz).  Prints one JSON object: per workload the medians
over the traced decisions of each phase's first start / last end relative to K1's first
start, each role's block durations, and the gaps between the kernels.

    ESC_LIB_PATH=escalator_amd/libescalator_hip_measure.so ESC_TAIL_TRACE=1 python scripts/tail_trace.py
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import escalator_amd as esc  # noqa: E402
from escalator_amd import _lib as L  # noqa: E402

ROLES = ["pieces", "tracker", "fold", "ordering"]


def tail_trace(ctx):
    lib = ctx.lib
    lib.esc_debug_tail_trace.restype = C.c_int32
    lib.esc_debug_tail_trace.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_int64, C.POINTER(C.c_int64)]
    n = C.c_int64(0)
    buf = np.zeros(1 << 22, np.uint64)
    L.check(lib.esc_debug_tail_trace(ctx.handle, buf.ctypes.data_as(C.POINTER(C.c_uint64)), buf.size, C.byref(n)))
    nt, nn = int(buf[0]), int(buf[1])
    t = buf[2:2 + 3 * nt].reshape(nt, 3).astype(np.int64)
    g = buf[2 + 3 * nt:2 + 3 * nt + 2 * nn].reshape(nn, 2).astype(np.int64)
    return t, g


def one(P, shard):
    N, G = 1_000_000, 10_000
    lo, hi = (0, P) if shard == 1 else (0, -(-P // shard))
    s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, p_lo=lo, p_hi=hi, threads=16)
    ctx = esc.Context(s, rank=0, world=shard)
    ctx.load_synth(s, pod_offset=lo, replicas=2 if shard == 1 else 8)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(4, 256)
    ctx.use_graph(False)
    ctx.k1_calibrate(16)

    def step():
        if shard == 1:
            ctx.run()
        else:
            ctx.reduce()
            ctx.decide()
        ctx.sync()

    for _ in range(5):
        step()
    rows = []
    for _ in range(20):
        step()
        k1 = ctx.k1_trace().astype(np.int64)
        t, g = tail_trace(ctx)
        t0 = k1[:, 0].min()
        r = {"k1_end": k1[:, 3].max() - t0, "tail_start": t[:, 0].min() - t0, "tail_end": t[:, 1].max() - t0,
             "ng_start": g[:, 0].min() - t0 if len(g) else 0, "ng_end": g[:, 1].max() - t0 if len(g) else 0}
        for k, name in enumerate(ROLES):
            m = t[:, 2] == k
            if m.any():
                d = t[m, 1] - t[m, 0]
                r[name + "_blocks"] = int(m.sum())
                r[name + "_first_start"] = t[m, 0].min() - t0
                r[name + "_last_end"] = t[m, 1].max() - t0
                r[name + "_dur_median"] = float(np.median(d))
                r[name + "_dur_max"] = int(d.max())
        if len(g):
            d = g[:, 1] - g[:, 0]
            r["ng_blocks"] = len(g)
            r["ng_dur_median"] = float(np.median(d))
            r["ng_dur_max"] = int(d.max())
        rows.append(r)
    keys = sorted(set().union(*rows))
    med = {k: float(np.median([r[k] for r in rows if k in r])) * (0.01 if not k.endswith("_blocks") else 1) for k in keys}
    med["unit"] = "us (100 MHz s_memrealtime ticks x 0.01), medians over 20 decisions, relative to K1's first start"
    med["gap_k1_tail"] = med["tail_start"] - med["k1_end"]
    med["gap_tail_ng"] = med["ng_start"] - med["tail_end"]
    return med


def main():
    assert os.environ.get("ESC_TAIL_TRACE") == "1", "set ESC_TAIL_TRACE=1 (and ESC_LIB_PATH to the measurement library)"
    out = {"config4": one(100_000_000, 1), "shard8": one(100_000_000, 8)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
