#!/usr/bin/env python3
"""Per-kernel summary of the TIMED launches of a bench.py run under rocprofv3.

    python scripts/prof_summary.py --trace T.csv [--fetch F.csv --write W.csv] \
        --last 30 --bench bench.json --out summary.json

A bench.py run launches K1 (k_pod_reduce) outside its timed region too: the share
calibration (esc_k1_calibrate, 16 rounds of decisions) and the warm-up steps.  bench.py's
roofline times K1 LAST, as 50 back-to-back launches between two HIP events (esc_k1_time),
so `--last 50` keeps exactly those K1 launches (by Dispatch_Id); for the other decision
kernels the last `--last` launches are the timed steps and the per-stage timing steps.
Kept launches feed:
  - the kernel trace (--trace, run_kernel_trace.csv of `rocprofv3 --kernel-trace`): mean and
    median duration per launch;
  - the PMC passes (--fetch / --write, run_counter_collection.csv of separate `--pmc
    FETCH_SIZE` and `--pmc WRITE_SIZE` runs of the same command): HBM bytes per launch as
    /opt/skills/guides/MI355X_MICROARCH.md § HBM prescribes (FETCH_SIZE is KiB and reports
    half the bytes of wide coalesced streaming reads on gfx950: read = 2 x 1024 x FETCH_SIZE;
    WRITE_SIZE KiB as is).
With --bench (the JSON line of the same command without the profiler), K1's algorithmic
bytes per launch and the bench's HIP-event launch time are set beside rocprof's, and the
fraction of the 8 TB/s peak is computed from both.
"""
import argparse
import collections
import csv
import json
import os
import statistics

PEAK_GBS = 8000.0
ORDER_KERNELS = ("k_ord_split", "k_ord_packed")
STEP_KERNELS = ("k_pod_reduce", "k_pod_bigtiles", "k_step_tail", "k_ord_split", "k_ord_packed", "k_node_groups")


def ours(k):
    """The library's kernels (every one is named k_*)."""
    return k.startswith("k_")


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].replace("esc::", "")


def last_dispatches(rows, n):
    """rows: (dispatch_id, value) per launch of one kernel -> the values of the last n launches."""
    rows = sorted(rows)
    return [v for _, v in rows[-n:]] if n > 0 else [v for _, v in rows]


def trace_summary(path, n):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if ours(k):
            per[k].append((int(r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for k, rows in per.items():
        d = last_dispatches(rows, n)
        out[k] = {"launches_total": len(rows), "launches_used": len(d), "mean_ns": statistics.mean(d),
                  "median_ns": statistics.median(d), "min_ns": min(d), "max_ns": max(d)}
    return out


def counter_summary(path, counter, n):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        if ours(k):
            per[k].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    return {k: (len(rows), last_dispatches(rows, n)) for k, rows in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--last", type=int, default=30)
    ap.add_argument("--bench")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"source": {k: v for k, v in vars(a).items() if v is not None}, "kernels": trace_summary(a.trace, a.last)}
    if a.fetch:
        for k, (tot, v) in counter_summary(a.fetch, "FETCH_SIZE", a.last).items():
            e = res["kernels"].setdefault(k, {})
            e.update(pmc_launches_total=tot, pmc_launches_used=len(v), fetch_kib=statistics.mean(v),
                     hbm_read_bytes=2 * 1024 * statistics.mean(v))
    if a.write:
        for k, (tot, v) in counter_summary(a.write, "WRITE_SIZE", a.last).items():
            e = res["kernels"].setdefault(k, {})
            e.update(write_kib=statistics.mean(v), hbm_write_bytes=1024 * statistics.mean(v))
    for e in res["kernels"].values():
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
    b = json.load(open(a.bench)) if a.bench else None
    if b and b["metric"].startswith("config5"):
        # config 5: the per-decision ordering kernels of the cold (cache-flushed) decisions
        # bench.py times last (--last = its steps + the final sort); bytes = the bench line's
        # roofline bytes per decision (8 B moved per membership; its bytes_8d: §8(d)'s 12 B)
        ks = [k for k in ORDER_KERNELS if k in res["kernels"]]
        t_ns = sum(res["kernels"][k]["mean_ns"] for k in ks)
        algo = b["roofline"]["bytes_per_decision"]
        hb = [res["kernels"][k].get("hbm_bytes") for k in ks]
        res["order"] = {"kernels": ks, "algorithmic_bytes_per_decision": algo, "rocprof_ns_per_decision": t_ns,
                        "rocprof_frac": algo / (t_ns * 1e-9) / 1e9 / PEAK_GBS if t_ns else None,
                        "bench_ms": b["ms_per_step"], "bench_frac": b["roofline"]["frac"],
                        "traffic_bytes": sum(hb) if all(x is not None for x in hb) and hb else None}
        if res["order"]["traffic_bytes"]:
            res["order"]["traffic_over_algorithmic"] = res["order"]["traffic_bytes"] / algo
        b = None
    if b and b.get("step_bytes"):
        # the whole decision step: every kernel one step launches, its PMC bytes against the
        # bench line's algorithmic bytes of the step (K1 pods + K2 node entries + orderings)
        ks = [k for k in STEP_KERNELS if k in res["kernels"]]
        hb = [res["kernels"][k].get("hbm_bytes") for k in ks]
        algo = b["step_bytes"]["total"]
        res["step"] = {"kernels": ks, "rocprof_ns": sum(res["kernels"][k]["mean_ns"] for k in ks),
                       "algorithmic_bytes": algo, "bench_ms_per_step": b["ms_per_step"],
                       "traffic_bytes": sum(hb) if hb and all(x is not None for x in hb) else None}
        if res["step"]["traffic_bytes"]:
            res["step"]["traffic_over_algorithmic"] = res["step"]["traffic_bytes"] / algo
    if b:
        rf = b["roofline"]
        k1 = res["kernels"].get("k_pod_reduce", {})
        algo = rf["algorithmic_bytes_per_launch"]
        res["k1"] = {
            "algorithmic_bytes_per_launch": algo,
            "bench_launch_ms": rf["launch_ms"],
            "bench_frac": rf["frac"],
            "rocprof_mean_ms": k1.get("mean_ns", 0) / 1e6,
            "rocprof_frac": algo / (k1["mean_ns"] * 1e-9) / 1e9 / PEAK_GBS if k1.get("mean_ns") else None,
            "rocprof_vs_bench": (k1.get("mean_ns", 0) / 1e6) / rf["launch_ms"] if rf["launch_ms"] else None,
            "traffic_bytes": k1.get("hbm_bytes"),
            "traffic_over_algorithmic": k1["hbm_bytes"] / algo if k1.get("hbm_bytes") else None,
            "bench_ms_per_step": b["ms_per_step"],
        }
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res.get("k1", res.get("order", {}))))
    for k, e in sorted(res["kernels"].items()):
        print(k, {x: (round(y, 1) if isinstance(y, float) else y) for x, y in e.items()})


if __name__ == "__main__":
    main()
