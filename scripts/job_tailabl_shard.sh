#!/bin/bash
# k_step_tail role ablations (timing only, wrong results) on rank 0's shard of an N=8 run:
# 8 no fold, 16 no node pieces (K2), 32 no packed orderings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-tailabl_shard}
mkdir -p $OUT
for A in 0 8 16 32 24 56; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python bench.py --shard-of 8 --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_shard8_a$A.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
done
echo done
