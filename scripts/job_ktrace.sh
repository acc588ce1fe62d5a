#!/bin/bash
# rocprofv3 kernel trace (timestamps) of the rank-0-of-8 shard step and the config-4 step:
# per-kernel durations and the gaps between consecutive kernels (scripts/timeline.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_ktrace}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for pair in "shard8:--shard-of 8" "full:"; do
    name=${pair%%:*}; args=${pair#*:}
    echo "[job] $(date) kernel trace $name"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run \
        -- python3 bench.py $args --steps 30 --warmup 5 --no-cpu-baseline --no-host --no-parity > $OUT/kt_$name.log 2>&1 || exit 1
    find $OUT/kt_$name -name "*kernel_trace.csv" -exec mv {} $OUT/kernel_trace_$name.csv \;
    find $OUT/kt_$name -name "*kernel_stats.csv" -exec mv {} $OUT/kernel_stats_$name.csv \;
    rm -rf $OUT/kt_$name
done
echo "[job] $(date) done"
