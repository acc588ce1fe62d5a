#!/bin/bash
# K5 (config 5): bench, kernel-trace summary and HBM PMC of the per-decision ordering kernels
# and of the age-index build kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_k5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) bench config 5"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; exit 1; }
cut -c1-1200 $OUT/bench5.json
echo "[job] $(date) kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run \
    -- python3 bench.py --config 5 --steps 20 --warmup 5 > $OUT/kt.log 2>&1 || exit 1
find $OUT/kt -name "*kernel_stats.csv" -exec mv {} $OUT/kernel_stats5.csv \;
rm -rf $OUT/kt
S="k_ord_count|k_ord_scatter|k_ord_packed|k_rs_hist|k_rs_scatter|k_memb_keys|k_memb_count|k_region_write"
for c in FETCH_SIZE:fetch WRITE_SIZE:write; do
    echo "[job] $(date) pmc ${c%%:*}"
    timeout -s KILL 120 rocprofv3 --pmc ${c%%:*} --kernel-include-regex "$S" --output-format csv \
        -d $OUT/pmc5_${c#*:} -o run -- python3 bench.py --config 5 --steps 3 --warmup 1 > $OUT/pmc5_${c#*:}.log 2>&1 || exit 1
    f=$(find $OUT/pmc5_${c#*:} -name "*counter_collection.csv" | head -1); [ -n "$f" ] && cp "$f" $OUT/pmc5_${c#*:}.csv
done
echo "[job] $(date) done"
