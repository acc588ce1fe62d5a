#!/bin/bash
# k_step_tail role ablations (timing only) at shard size and full size.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-tailabl}
mkdir -p $OUT
for P in 12500000 100000000; do
  for A in 0 8 16 32 24 40 48 1; do
    ESC_K3_ABLATE=$A timeout -k 10 240 python bench.py --pods $P --steps 30 --warmup 5 --no-cpu-baseline --no-parity > $OUT/bench_p${P}_a$A.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
  done
done
echo done
