#!/bin/bash
# One-stream step (K1, k_step_tail, k_node_groups): GPU suite, benches, config 5, timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-tail}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
     > $OUT/bench_p12.5M.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
timeout -k 10 300 python bench.py --config 5 > $OUT/bench5.json 2> $OUT/b5.err || { tail $OUT/b5.err; exit 1; }
for P in 12500000 100000000; do
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr_$P -o run \
    -- python3 bench.py --pods $P --steps 20 --warmup 5 --no-cpu-baseline --no-parity > $OUT/tr_$P.log 2>&1 || exit 1
find $OUT/tr_$P -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace_p$P.csv \;
rm -rf $OUT/tr_$P
done
echo done
