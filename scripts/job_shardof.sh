#!/bin/bash
# Per-rank device time of an N=W config-4 run, measured on one GPU (bench --shard-of W).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-shardof}
mkdir -p $OUT
for W in 2 4 8; do
  timeout -k 10 240 python bench.py --shard-of $W --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench_shard$W.json 2> $OUT/s$W.err || { tail $OUT/s$W.err; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof8.log 2>&1 || { tail $GRAFT_REPO_ROOT/$OUT/prof8.log; exit 1; }
echo done
