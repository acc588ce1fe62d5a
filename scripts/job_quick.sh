#!/bin/bash
# Quick GPU check: the GPU suite (optionally filtered by K=...), the default bench and the
# 12.5M-pod shard-size bench with a kernel-trace summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
    > $OUT/bench_p12.5M.json 2> $OUT/bench_p12.5M.err || { tail $OUT/bench_p12.5M.err; exit 1; }
cat $OUT/bench_p12.5M.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p12 -o run \
    -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/prof_p12.log 2>&1 || exit 1
find $OUT/prof_p12 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_p12.csv \;
rm -rf $OUT/prof_p12
echo done
