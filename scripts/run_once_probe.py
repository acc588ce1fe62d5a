"""Where the config-4 RunOnce goes (the bench's `run_once`): the median wall time of each
C-ABI call of the Go shim's RunOnce on the resident snapshot — esc_set_state, esc_step +
esc_sync, esc_results (every group), esc_selections (sizes), esc_selections (nodes).

    python scripts/run_once_probe.py > out.json
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import escalator_amd as esc  # noqa: E402
from escalator_amd import _lib as L  # noqa: E402
from escalator_amd.context import DECISION_DTYPE, TOTALS_DTYPE  # noqa: E402


def main():
    s = esc.Synth(100_000_000, 1_000_000, 10_000, config=4, seed=0xE5CA1A7E00000004, threads=16)
    ctx = esc.Context(s)
    ctx.load_synth(s, replicas=2)
    ctx.set_state(s.states)
    ctx.set_order_in_step(True)
    ctx.set_selections(4, 256)
    ctx.k1_calibrate(16)
    lib, h, G = ctx.lib, ctx.handle, ctx.G
    tot, dec = np.zeros(G, TOTALS_DTYPE), np.zeros(G, DECISION_DTYPE)
    which, off = np.zeros(G, np.int32), np.zeros(G + 1, np.int64)
    idx = np.zeros(G * 257, np.int64)
    tp, dp = tot.ctypes.data_as(C.POINTER(L.GroupTotals)), dec.ctypes.data_as(C.POINTER(L.GroupDecision))
    wp, op, ip = (which.ctypes.data_as(C.POINTER(C.c_int32)), off.ctypes.data_as(C.POINTER(C.c_int64)),
                  idx.ctypes.data_as(C.POINTER(C.c_int64)))
    n = C.c_int64()
    calls = [("esc_set_state", lambda: lib.esc_set_state(h, ctx._state)),
             ("esc_step", lambda: lib.esc_step(h)),
             ("esc_sync", lambda: lib.esc_sync(h)),
             ("esc_results", lambda: lib.esc_results(h, tp, dp)),
             ("esc_selections_sizes", lambda: lib.esc_selections(h, wp, op, None, 0, C.byref(n))),
             ("esc_selections_nodes", lambda: lib.esc_selections(h, wp, op, ip, len(idx), C.byref(n)))]
    t = {k: [] for k, _ in calls}
    tot_ms = []
    for rep in range(40):
        t0 = time.perf_counter()
        for k, f in calls:
            a = time.perf_counter()
            L.check(f(), k)
            t[k].append((time.perf_counter() - a) * 1e3)
        tot_ms.append((time.perf_counter() - t0) * 1e3)
    out = {k: float(np.median(v[5:])) for k, v in t.items()}
    out["run_once"] = float(np.median(tot_ms[5:]))
    out["unit"] = "ms, median of 35 (config 4: 100 M pods / 1 M nodes / 10 k groups, selections slack 4)"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
