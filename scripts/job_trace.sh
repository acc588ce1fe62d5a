#!/bin/bash
# GPU suite, config-5 bench (K5 classify reads flags only), K1 per-workgroup timelines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/trace
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --config 5 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; exit 1; }
PODS=12500000 VARIANTS=0,6 timeout -k 10 200 python -u scripts/k1_trace.py > $OUT/trace_p12.5M.json 2> $OUT/t12.err || { tail $OUT/t12.err; exit 1; }
PODS=100000000 VARIANTS=0,6 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/trace_p100M.json 2> $OUT/t100.err || { tail $OUT/t100.err; exit 1; }
echo done
