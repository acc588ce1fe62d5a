#!/bin/bash
# Quick state check: GPU suite, default bench (config 4) and the rank-0-of-8 shard bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
echo "[job] $(date) bench"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 240 python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
    > $OUT/bench_shard8.json 2> $OUT/bench_shard8.err || { tail $OUT/bench_shard8.err; exit 1; }
cat $OUT/bench_shard8.json
echo "[job] $(date) done"
