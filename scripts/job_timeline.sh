#!/bin/bash
# Per-dispatch kernel timeline of the decision step (rocprofv3 kernel trace, no counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-timeline}
mkdir -p $OUT
export TMPDIR=/tmp
for P in 12500000 100000000; do
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$P -o run \
    -- python3 bench.py --pods $P --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/tr_$P.log 2>&1 || exit 1
find $OUT/tr_$P -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace_p$P.csv \;
rm -rf $OUT/tr_$P
done
echo done
