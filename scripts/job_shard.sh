#!/bin/bash
# Shard-size step measurements (12.5M pods = one rank's share at N=8): zero-copy on/off,
# plus a rocprofv3 kernel trace of the default step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/shard
export TMPDIR=/tmp
for zc in 0 1; do
  ESC_NO_ZEROCOPY=$zc timeout -k 10 180 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
     > gpurun_out/shard/bench_p12.5M_nozc$zc.json 2> gpurun_out/shard/bench_p12.5M_nozc$zc.err || exit 1
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/shard/prof -o run -- python3 bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity \
     > gpurun_out/shard/bench_prof.json 2> gpurun_out/shard/bench_prof.err || exit 1
find gpurun_out/shard/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/shard/kernel_stats.csv \;
echo done
