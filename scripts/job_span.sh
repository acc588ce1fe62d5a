#!/bin/bash
# K2 spans in the step tail: GPU suite, benches (direct enqueue), role ablations, timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-span}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
for A in 0 40 48; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M_a$A.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run \
    -- python3 bench.py --pods 12500000 --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/tr.log 2>&1 || exit 1
find $OUT/tr -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace_p12.5M.csv \;
rm -rf $OUT/tr
echo done
