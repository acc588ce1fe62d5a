#!/bin/bash
# Round check: GPU suite, smoke, default bench (config 4), shard-size bench, config 5,
# and rocprofv3 kernel-trace summaries of the bench commands.  Each GPU step has its own
# time limit; the first failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
STEPS=${STEPS:-20}
echo "[job] $(date) pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "[job] $(date) smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
echo "[job] $(date) bench"
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
    > $OUT/bench_p12.5M.json 2> $OUT/bench_p12.5M.err || { tail $OUT/bench_p12.5M.err; exit 1; }
cat $OUT/bench_p12.5M.json
timeout -k 10 300 python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
    > $OUT/bench_shard8.json 2> $OUT/bench_shard8.err || { tail $OUT/bench_shard8.err; exit 1; }
cut -c1-600 $OUT/bench_shard8.json
echo "[job] $(date) config 5"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; exit 1; }
cat $OUT/bench5.json
echo "[job] $(date) rocprofv3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-parity > $OUT/prof.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p12 -o run \
    -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/prof_p12.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o run \
    -- python3 bench.py --config 5 --steps 20 --warmup 3 > $OUT/prof5.log 2>&1 || exit 1
for d in prof prof_p12 prof5; do
    find $OUT/$d -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_$d.csv \;
    rm -rf $OUT/$d/*/*_kernel_trace.csv 2>/dev/null
done
echo "[job] $(date) done"
