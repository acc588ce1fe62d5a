#!/bin/bash
# K1 dynamic tail: GPU suite, benches at 100M / 12.5M with the tail (default) and without
# (ESC_K1_STATIC=1), per-workgroup timelines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-dyn}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for sf in ${FRACS:-0.8 1.0}; do
  ESC_K1_STATIC=$sf timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_s$sf.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  ESC_K1_STATIC=$sf timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
     > $OUT/bench_p12.5M_s$sf.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
done
ESC_K1_STATIC=0.8 PODS=12500000 VARIANTS=0 timeout -k 10 200 python -u scripts/k1_trace.py > $OUT/trace_p12.5M.json 2> $OUT/t12.err || { tail $OUT/t12.err; exit 1; }
ESC_K1_STATIC=0.8 PODS=100000000 VARIANTS=0 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/trace_p100M.json 2> $OUT/t100.err || { tail $OUT/t100.err; exit 1; }
echo done
