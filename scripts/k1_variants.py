"""Times the K1 (k_pod_reduce) variants on one snapshot, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24), and checks every variant's totals are identical."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

cfg = int(os.environ.get("CFG", 4))
P, N, G = {4: (100_000_000, 1_000_000, 10_000), 2: (1_000_000, 10_000, 100), 3: (10_000_000, 100_000, 100)}[cfg]
P = int(os.environ.get("PODS", P))            # a rank's shard at N > 1 (fixed-cost study)
variants = [int(v) for v in os.environ.get("VARIANTS", "0,2,9,10,11").split(",")]
rounds = int(os.environ.get("ROUNDS", 3))
import escalator_amd as esc  # noqa: E402

s = esc.Synth(P, N, G, config=cfg, seed=0xE5CA1A7E00000000 + cfg, threads=16)
from escalator_amd import layout  # noqa: E402
from oracle import soa
bytes_k1 = layout.pod_bytes(s.pods(), len(soa.group_tables(s.groups)["pair_ids"]))
ctxs = {}
for v in variants:
    os.environ["ESC_K1_VARIANT"] = str(v)
    c = esc.Context(s)
    c.load_synth(s, replicas=1 if cfg == 4 else 8)
    c.set_state(s.states)
    if os.environ.get("CALIBRATE", "0") != "0":      # calibrated shares (as the bench runs K1)
        c.k1_calibrate(int(os.environ["CALIBRATE"]))
    c.set_timing(True)
    ctxs[v] = c
res = {v: [] for v in variants}
ref = None
for r in range(rounds):
    for v in variants:
        c = ctxs[v]
        for _ in range(5):
            c.run()
            c.sync()
            res[v].append(c.stage_times()[0])
        t, d = c.results()
        if v >= 9:
            continue                          # ablation: timing only
        if ref is None:
            ref = (t.tobytes(), d.tobytes())
        assert (t.tobytes(), d.tobytes()) == ref, "variant %d differs" % v
out = {}
for v in variants:
    ms = np.array(res[v])
    out[v] = {"median_ms": float(np.median(ms)), "min_ms": float(ms.min()),
              "GBps_median": bytes_k1 / (np.median(ms) * 1e-3) / 1e9}
print(json.dumps({"config": cfg, "pods": P, "k1_bytes": int(bytes_k1), "variants": out}))
