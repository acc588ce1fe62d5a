#!/bin/bash
# GPU suite + benches at full and shard size + fold/decide ablations + kernel traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=${TAG:-kb}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
B="python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity"
timeout -k 10 240 $B > $OUT/bench_p12.5M.json 2> $OUT/p12.err || { tail $OUT/p12.err; exit 1; }
ESC_K3_ABLATE=1 timeout -k 10 240 $B > $OUT/bench_p12.5M_k3abl1.json 2> $OUT/p12a.err || { tail $OUT/p12a.err; exit 1; }
ESC_NO_ZEROCOPY=1 timeout -k 10 240 $B > $OUT/bench_p12.5M_nozc.json 2> $OUT/p12z.err || { tail $OUT/p12z.err; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_p12 -o run \
    -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/prof_p12.log 2>&1 || exit 1
find $OUT/prof_p12 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_p12.csv \;
rm -rf $OUT/prof_p12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run \
    -- python3 bench.py --no-cpu-baseline --no-parity > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/prof
echo done
