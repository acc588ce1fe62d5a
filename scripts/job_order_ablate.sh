#!/bin/bash
# k_ord_fused ablations (timing only, ESC_ORDER_ABLATE: 1 no look-back, 2 no scatter,
# 4 block id instead of the ticket) and chunk sizes (ESC_ORDER_CHUNK) under rocprofv3
# kernel trace; prints each run's K5 per-decision kernel average durations (us).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CFGS:-"16384 0" "16384 3" "16384 7" "8192 0" "4096 0" "4096 3"}; do
    set -- $cfg
    tag=ord_c$1_a$2
    ESC_ORDER_CHUNK=$1 ESC_ORDER_ABLATE=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/$tag -o run -- python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/$tag.log 2>&1 || exit 1
    python3 - "$tag" <<'PY'
import csv, sys
t = sys.argv[1]
for r in csv.DictReader(open("gpurun_out/%s/run_kernel_stats.csv" % t)):
    if "k_ord" in r["Name"]:
        print(t, r["Name"][:30], "calls", r["Calls"], "avg_us %.1f" % (float(r["AverageNs"]) / 1e3))
PY
done
