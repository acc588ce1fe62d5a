#!/bin/bash
# Graph replay vs direct kernel enqueue for back-to-back decisions; timeline of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-graph}
mkdir -p $OUT
export TMPDIR=/tmp
for P in 12500000 100000000; do
  for G in "" "--no-graph"; do
    timeout -k 10 240 python bench.py --pods $P --steps 50 --warmup 10 --no-cpu-baseline --no-parity $G > $OUT/bench_p${P}${G}.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run \
    -- python3 bench.py --pods 12500000 --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-graph > $OUT/tr.log 2>&1 || exit 1
find $OUT/tr -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace_p12.5M_nograph.csv \;
rm -rf $OUT/tr
echo done
