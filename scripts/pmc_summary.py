#!/usr/bin/env python3
"""Summarises the rocprofv3 --pmc passes of scripts/pmc_job.sh into one JSON per round.

    python scripts/pmc_summary.py <pmc_dir_prefix> <out.json>

e.g. `python scripts/pmc_summary.py gpurun_out/pmc_r01c profiles/r01_v2/pmc_summary.json` reads
gpurun_out/pmc_r01c_{fetch,write,sq,lds}/run_counter_collection.csv.

HBM bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md § HBM [CDNA4]:
FETCH_SIZE is in KiB and reports half the bytes of wide coalesced streaming reads on
gfx950, so read bytes = 2 x 1024 x FETCH_SIZE; WRITE_SIZE (KiB) is taken as is.
SQ_* wave counters are in quad-cycles; only their ratios are reported."""
import collections
import csv
import json
import os
import sys


def load(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return d
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    pre, out = sys.argv[1], sys.argv[2]
    merged = collections.defaultdict(dict)
    for tag in ("fetch", "write", "sq", "lds", "occ"):
        for k, cs in load(f"{pre}_{tag}/run_counter_collection.csv").items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
                merged[k]["launches"] = len(v)
    res = {}
    for k, c in merged.items():
        e = {"launches": c.get("launches")}
        if "FETCH_SIZE" in c:
            e["fetch_kib_raw"] = c["FETCH_SIZE"]
            e["hbm_read_bytes"] = 2 * 1024 * c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            e["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
        if "hbm_read_bytes" in e and "hbm_write_bytes" in e:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            e["wait_any_frac"] = c.get("SQ_WAIT_ANY", 0) / wc
            e["wait_inst_any_frac"] = c.get("SQ_WAIT_INST_ANY", 0) / wc
            e["active_frac"] = 1 - e["wait_any_frac"] - e["wait_inst_any_frac"]
        if c.get("SQ_WAVES"):
            for name in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD"):
                if name in c:
                    e[name.lower() + "_per_wave"] = c[name] / c["SQ_WAVES"]
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        e["raw"] = c
        res[k] = e
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, e in res.items():
        print(k, {a: b for a, b in e.items() if a != "raw"})


if __name__ == "__main__":
    main()
