#!/bin/bash
# K1 change check: the K1 / synthetic parity tests, the default and rank-0-of-8 benches,
# a kernel-trace summary and the HBM PMC passes of the rank-0-of-8 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_k1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest (K1 subset)"
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "synthetic or k1 or config4 or multi_device_context or step_graph or big_tiles or random_objects or determinism" \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "[job] $(date) bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 240 python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
    > $OUT/bench_shard8.json 2> $OUT/bench_shard8.err || { tail $OUT/bench_shard8.err; exit 1; }
cat $OUT/bench_shard8.json
echo "[job] $(date) rocprofv3 kernel trace (shard 8)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof8 -o run \
    -- python3 bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline > $OUT/prof8.log 2>&1 || exit 1
find $OUT/prof8 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_shard8.csv \;
rm -rf $OUT/prof8
K="k_pod_reduce|k_step_tail|k_node_groups|k_decide"
CMD="python3 bench.py --shard-of 8 --steps 3 --warmup 1 --no-cpu-baseline"
for pass in FETCH_SIZE WRITE_SIZE; do
    echo "[job] $(date) pmc $pass"
    timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "$K" --output-format csv \
        -d $OUT/pmc_$pass -o run -- $CMD > $OUT/pmc_$pass.log 2>&1 || exit 1
    find $OUT/pmc_$pass -name "*counter_collection.csv" -exec cp {} $OUT/pmc_${pass}.csv \;
    rm -rf $OUT/pmc_$pass
done
echo "[job] $(date) done"
