#!/bin/bash
# GPU suite, then the default bench and the shard-size (12.5M pods) bench with a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-step}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
timeout -k 10 240 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M.json 2> $OUT/bench_p12.5M.err || exit 1
ESC_NO_ZEROCOPY=1 timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M_nozc.json 2> $OUT/bench_p12.5M_nozc.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_prof.json 2> $OUT/bench_prof.err || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_p12.5M.csv \;
rm -rf $OUT/prof
echo done
