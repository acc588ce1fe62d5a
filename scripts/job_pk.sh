#!/bin/bash
# Packed K blocks: GPU suite, config 4 + rank-0-of-8 benches for K1_PK_DS variants
# (ESC_LIB_PATH), kernel-trace summary and HBM PMC passes of the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_pk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then unset ESC_LIB_PATH; else export ESC_LIB_PATH=$PWD/escalator_amd/libescalator_hip_$v.so; fi
    echo "[job] $(date) bench $v"
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host > $OUT/bench_$v.json 2> $OUT/bench_$v.err || { tail $OUT/bench_$v.err; exit 1; }
    timeout -k 10 240 python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
        > $OUT/bench_shard8_$v.json 2> $OUT/bench_shard8_$v.err || { tail $OUT/bench_shard8_$v.err; exit 1; }
    python - $OUT/bench_$v.json $OUT/bench_shard8_$v.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f)); r = d["roofline"]
    print(f, "step %.4f ms  K1 %.4f ms frac %.3f" % (d["ms_per_step"], r["launch_ms"], r["frac"]), d["stage_ms"])
PY
done
unset ESC_LIB_PATH
[ -n "$NO_PROF" ] && exit 0
echo "[job] $(date) rocprofv3 kernel trace (config 4)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
K="k_pod_reduce|k_step_tail|k_node_groups|k_decide"
for pair in "full:python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host --no-parity" \
            "shard8:python3 bench.py --shard-of 8 --steps 3 --warmup 1 --no-cpu-baseline"; do
    name=${pair%%:*}; cmd=${pair#*:}
    for c in FETCH_SIZE:fetch WRITE_SIZE:write; do
        echo "[job] $(date) pmc $name ${c%%:*}"
        timeout -s KILL 120 rocprofv3 --pmc ${c%%:*} --kernel-include-regex "$K" --output-format csv \
            -d $OUT/pmc_${name}_${c#*:} -o run -- $cmd > $OUT/pmc_${name}_${c#*:}.log 2>&1 || exit 1
        find $OUT/pmc_${name}_${c#*:} -name "*counter_collection.csv" -exec mv {} $OUT/pmc_${name}_${c#*:}/run_counter_collection.csv \;
    done
done
echo "[job] $(date) done"
