#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-k2abl}
mkdir -p $OUT
for A in 0 40; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M_a$A.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
done
echo done
