#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-quick2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
timeout -k 10 240 python bench.py --pods 12500000 --steps 50 --warmup 10 --no-cpu-baseline --no-parity > $OUT/bench_p12.5M.json 2> $OUT/p.err || { tail $OUT/p.err; exit 1; }
echo done
