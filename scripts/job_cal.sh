#!/bin/bash
# K1 share calibration: GPU suite, benches (calibrated in bench.py), per-workgroup timelines
# after calibration, kernel traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-cal}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
     > $OUT/bench_p12.5M.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
CALIBRATE=16 PODS=12500000 VARIANTS=0 timeout -k 10 200 python -u scripts/k1_trace.py > $OUT/trace_p12.5M.json 2> $OUT/t12.err || { tail $OUT/t12.err; exit 1; }
CALIBRATE=16 PODS=100000000 VARIANTS=0 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/trace_p100M.json 2> $OUT/t100.err || { tail $OUT/t100.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p12 -o run \
    -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/prof_p12.log 2>&1 || exit 1
find $OUT/prof_p12 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_p12.csv \;
rm -rf $OUT/prof_p12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --no-cpu-baseline --no-parity > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
echo done
