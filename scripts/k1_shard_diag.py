"""K1 per-workgroup diagnostics at a rank's shard (rank 0 of W, as bench.py --shard-of W):
per workgroup its XCD, K weight, class runs, start / K-phase / end times over several
decisions, before and after the share calibration (esc_k1_calibrate).

    SHARD_OF=8 [CAL_MORE=32,32] python scripts/k1_shard_diag.py > out.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import escalator_amd as esc  # noqa: E402
from escalator_amd.dist import shard_range  # noqa: E402

W = int(os.environ.get("SHARD_OF", 8))
P, N, G = 100_000_000, 1_000_000, 10_000
lo, hi = shard_range(P, 0, W)
s = esc.Synth(P, N, G, config=4, seed=0xE5CA1A7E00000004, p_lo=lo, p_hi=hi, threads=16)
c = esc.Context(s, rank=0, world=W)
c.load_synth(s, pod_offset=lo, replicas=8)
c.set_state(s.states)
c.set_order_in_step(True)


def runs(k=10):
    out = []
    for _ in range(k):
        c.reduce()
        c.decide()
        c.sync()
        out.append(c.k1_trace().astype(np.int64))
    return out


def summarize(rs):
    t = []
    for r in rs:
        t0 = r[:, 0].min()
        t.append(np.stack([r[:, 0] - t0, r[:, 1] - r[:, 0], r[:, 3] - r[:, 1], r[:, 3] - t0], 1) * 0.01)
    t = np.array(t)                                  # [run, wg, (start, kphase, tail, end)] us
    r = rs[-1]
    return {"start_us": t[:, :, 0].mean(0).round(2).tolist(), "kphase_us": t[:, :, 1].mean(0).round(2).tolist(),
            "after_k_us": t[:, :, 2].mean(0).round(2).tolist(), "end_us": t[:, :, 3].mean(0).round(2).tolist(),
            "end_max_us_per_run": t[:, :, 3].max(1).round(2).tolist(),
            "xcc": (r[:, 5] & 0xF).tolist(), "runs": r[:, 6].tolist(), "kweight": r[:, 7].tolist()}


out = {"shard_of": W, "pods": hi - lo, "uncalibrated": summarize(runs())}
c.k1_calibrate(16)
out["calibrated"] = summarize(runs())
# CAL_MORE=32,32: further esc_k1_calibrate calls (continuing from the current shares)
for i, r in enumerate(x for x in os.environ.get("CAL_MORE", "").split(",") if x):
    c.k1_calibrate(int(r))
    out["calibrated_more_%d" % i] = summarize(runs())
c.set_timing(True)
st = []
for _ in range(10):
    c.reduce()
    c.decide()
    c.sync()
    st.append(c.stage_times())
c.set_timing(False)
out["stage_ms"] = np.mean(np.array(st), 0).round(5).tolist()
out["k1_time_ms"] = c.k1_time(50)
print(json.dumps(out))
