#!/bin/bash
# Reaping (K6/K7): GPU reaping tests, config-4 reaping bench, kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-reap}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python -u scripts/bench_reaping.py --steps 20 --warmup 3 > $OUT/bench_reaping.json 2> $OUT/br.err || { tail $OUT/br.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 scripts/bench_reaping.py --steps 20 --warmup 3 > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_reaping.csv \;
rm -rf $OUT/prof
echo done
