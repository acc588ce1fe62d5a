"""Per-call latency of the Go-signature drop-ins (esc_pods_requests_total,
esc_nodes_capacity_total) against the slice size: where the time of one call goes
(VERDICT r4 item 7).  Medians of 500 calls, ms; parity against the C oracle each size.

    python scripts/dropin_probe.py > out.json
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

s = esc.Synth(20_000, 2_000, 1, config=1, seed=0xE5CA1A7E00000001)
po, n_p, no, n_n = s.objects()
ctx = esc.Context(s.groups, device=0)
lib = ctx.lib
mem, cpu = C.c_int64(), C.c_int64()
out = {"pods": {}, "nodes": {}}
for n in (1, 50, 949, 4096, 20_000):
    arr = (L.PodObj * n)(*[po[i] for i in range(n)])
    L.check(lib.esc_pods_requests_total(ctx.handle, arr, n, C.byref(mem), C.byref(cpu)))
    ts = []
    for _ in range(500):
        t0 = time.perf_counter()
        lib.esc_pods_requests_total(ctx.handle, arr, n, C.byref(mem), C.byref(cpu))
        ts.append(time.perf_counter() - t0)
    out["pods"][n] = {"median_ms": float(np.median(ts)) * 1e3, "p90_ms": float(np.percentile(ts, 90)) * 1e3,
                      "cpu_m": cpu.value, "mem_b": mem.value}
for n in (1, 50, 2000):
    arr = (L.NodeObj * n)(*[no[i] for i in range(n)])
    ts = []
    for _ in range(500):
        t0 = time.perf_counter()
        lib.esc_nodes_capacity_total(ctx.handle, arr, n, C.byref(mem), C.byref(cpu))
        ts.append(time.perf_counter() - t0)
    out["nodes"][n] = {"median_ms": float(np.median(ts)) * 1e3, "p90_ms": float(np.percentile(ts, 90)) * 1e3}
# ctypes call floor: a host-only ABI call
ts = []
for _ in range(2000):
    t0 = time.perf_counter()
    lib.esc_abi_version()
    ts.append(time.perf_counter() - t0)
out["ctypes_floor_ms"] = float(np.median(ts)) * 1e3
print(json.dumps(out))
