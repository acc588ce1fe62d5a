"""K1 per-workgroup timeline (ESC_K1_TRACE=1 diagnostics): start skew, K-tile phase, C-tile
phase and flush per workgroup, the slowest workgroup vs the mean, per-XCD means.

    PODS=12500000 VARIANT=0 python scripts/k1_trace.py > out.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import escalator_amd as esc  # noqa: E402

P = int(os.environ.get("PODS", 12_500_000))
variants = [int(v) for v in os.environ.get("VARIANTS", "0").split(",")]
s = esc.Synth(P, 1_000_000, 10_000, config=4, seed=0xE5CA1A7E00000004, threads=16)
out = {"pods": P, "variants": {}}
for v in variants:
    os.environ["ESC_K1_VARIANT"] = str(v)
    c = esc.Context(s)
    c.load_synth(s, replicas=max(1, min(4, 1_000_000_000 // max(P * 24, 1))))
    c.set_state(s.states)
    c.use_graph(False)
    if os.environ.get("CALIBRATE", "0") != "0":
        c.k1_calibrate(int(os.environ["CALIBRATE"]))
    runs = []
    for k in range(12):
        c.run()
        c.sync()
        if k >= 2:
            runs.append(c.k1_trace().astype(np.int64))
    stats = []
    for tr in runs:
        t0 = tr[:, 0].min()
        st, kd, cd, fl = (tr[:, i] - t0 for i in range(4))
        stats.append({
            "kernel_us": float(fl.max()) * 0.01,                    # 100 MHz ticks -> us
            "start_skew_us": float(st.max()) * 0.01,
            "k_phase_us_mean": float((kd - st).mean()) * 0.01, "k_phase_us_max": float((kd - st).max()) * 0.01,
            "k_phase_us_min": float((kd - st).min()) * 0.01,
            "c_phase_us_mean": float((cd - kd).mean()) * 0.01, "c_phase_us_max": float((cd - kd).max()) * 0.01,
            "flush_us_mean": float((fl - cd).mean()) * 0.01, "flush_us_max": float((fl - cd).max()) * 0.01,
            "end_spread_us": float(fl.max() - fl.min()) * 0.01,
            "end_mean_us": float(fl.mean()) * 0.01,
        })
    agg = {k: float(np.median([x[k] for x in stats])) for k in stats[0]}
    # stability of the per-workgroup durations across decisions (is the imbalance a
    # property of the workgroup / CU, or noise?)
    dur = np.array([(r[:, 3] - r[:, 0]).astype(np.float64) for r in runs])
    cc = [float(np.corrcoef(dur[i], dur[i + 1])[0, 1]) for i in range(len(dur) - 1)]
    agg["dur_corr_consecutive"] = cc
    rel = dur / dur.mean(axis=1, keepdims=True)
    agg["dur_rel_std_per_wg_over_runs"] = float(rel.std(axis=0).mean())
    agg["dur_rel_spread_mean_over_runs"] = float(rel.mean(axis=0).max() - rel.mean(axis=0).min())
    agg["dur_rel_mean_per_wg"] = [round(float(x), 4) for x in rel.mean(axis=0)]
    agg["xcc_per_wg"] = [int(x) for x in (runs[-1][:, 5] & 0xF)]
    agg["hwid_per_wg"] = [int(x) for x in runs[-1][:, 4]]
    tr = runs[-1]
    t0 = tr[:, 0].min()
    xcc = (tr[:, 5] & 0xF).astype(int)
    per_xcc = {int(x): {"n": int((xcc == x).sum()),
                        "end_mean_us": float((tr[xcc == x, 3] - t0).mean()) * 0.01,
                        "k_phase_mean_us": float((tr[xcc == x, 1] - tr[xcc == x, 0]).mean()) * 0.01}
               for x in sorted(set(xcc))}
    # the cost of a class run: per-workgroup K phase ~ a + b * K weight + c * runs (least
    # squares over every workgroup of every decision); c is what a run's restart costs
    X, y = [], []
    for r in runs:
        ok = r[:, 6] > 0
        X.append(np.stack([np.ones(ok.sum()), r[ok, 7].astype(np.float64), r[ok, 6].astype(np.float64)], 1))
        y.append((r[ok, 1] - r[ok, 0]).astype(np.float64) * 0.01)
    if X and sum(len(v) for v in y) > 3:
        X, y = np.concatenate(X), np.concatenate(y)
        coef, *_ = np.linalg.lstsq(X, y, rcond=None)
        agg["k_phase_fit_us"] = {"intercept": float(coef[0]), "per_kweight_ns": float(coef[1] * 1e3),
                                 "per_run": float(coef[2])}
        agg["runs_hist"] = {int(k): int(v) for k, v in zip(*np.unique(runs[-1][:, 6], return_counts=True))}
        agg["k_phase_mean_by_runs"] = {int(k): float(y[X[:, 2] == k].mean()) for k in np.unique(X[:, 2])}
    order = np.argsort(tr[:, 3])
    agg["slowest_blocks"] = [int(b) for b in order[-8:]]
    agg["per_xcc_last_run"] = per_xcc
    agg["end_us_sorted_last_run_deciles"] = [float(np.percentile(tr[:, 3] - t0, q)) * 0.01 for q in range(0, 101, 10)]
    out["variants"][v] = agg
    del c
print(json.dumps(out))
