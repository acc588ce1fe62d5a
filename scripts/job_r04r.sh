#!/bin/bash
# Round 4: tail occupancy (162 -> 82 VGPRs: fold 4 wave-loads in flight, K2 spans of 256
# entries) — parity suite, then the steps and the role ablations at config 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04w}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k, v in d['stage_ms'].items()}, d.get('parity'))"; }
timeout -k 10 240 python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host > $OUT/shard8.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
show $OUT/shard8.json shard8
timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host > $OUT/full.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
show $OUT/full.json full
for A in 40 48 24 56; do
  ESC_K3_ABLATE=$A timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host --no-parity \
      > $OUT/tailabl_a$A.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
  show $OUT/tailabl_a$A.json "ablate $A"
done
echo "[job] $(date) done"
