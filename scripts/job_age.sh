#!/bin/bash
# Streaming age-index build: GPU suite, config 5 bench, kernel stats of the build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-age}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run \
    -- python3 bench.py --config 5 --steps 20 --warmup 3 > $OUT/prof5.log 2>&1 || exit 1
find $OUT/prof5 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_prof5.csv \;
rm -rf $OUT/prof5
echo done
