#!/bin/bash
# A/B of the fused K1 fold at shard size and full size: fused / separate fold, with and
# without the side stream (ESC_NO_FORK=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-fold_ab}
mkdir -p $OUT
for P in 12500000 100000000; do
  for F in 0 1; do
    for NF in 0 1; do
      ESC_FUSED_FOLD=$((1-F)) ESC_NO_FORK=$NF timeout -k 10 200 python bench.py --pods $P --steps 30 --warmup 5 \
          --no-cpu-baseline --no-parity > $OUT/p${P}_nofused${F}_nofork${NF}.json 2> $OUT/err.log || exit 1
      python -c "import json,sys; d=json.load(open('$OUT/p${P}_nofused${F}_nofork${NF}.json')); print('$P nofused=$F nofork=$NF', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k,v in d['stage_ms'].items()})"
    done
  done
done
