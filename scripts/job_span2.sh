#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-span2}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "step_graph or synthetic_vs or tracker or sharded" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for A in 0 40; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M_a$A.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
done
echo done
