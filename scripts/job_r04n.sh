#!/bin/bash
# Round 4: k_step_tail role ablations at config 4 (N = 1), timing only (ESC_K3_ABLATE:
# 8 no fold, 16 no node pieces, 32 no packed orderings, 64 no tracker blocks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 240 python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host > $OUT/shard8.json 2> $OUT/shard8.err || { tail $OUT/shard8.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/shard8.json')); print('shard8', round(d['ms_per_step']*1e3, 1), {k: round(v*1e3, 1) for k, v in d['stage_ms'].items()})"
for A in 0 8 16 32 64 24 40 48 56 120; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host --no-parity \
      > $OUT/tailabl_a$A.json 2> $OUT/tailabl.err || { tail $OUT/tailabl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/tailabl_a$A.json')); print('ablate $A', round(d['ms_per_step']*1e3, 1), {k: round(v*1e3, 1) for k, v in d['stage_ms'].items()})"
done
echo "[job] $(date) done"
