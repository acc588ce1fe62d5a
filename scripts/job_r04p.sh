#!/bin/bash
# Round 4: K2 span shape — pieces per span (ESC_SPAN_PIECES) against the tail's K2-alone time
# (ESC_K3_ABLATE=40) and the whole step, config 4 and the shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04p}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,1), {k: round(v*1e3,1) for k, v in d['stage_ms'].items()}, d.get('parity'))"; }
for SP in 63 16 8 4; do
  for A in 40 0; do
    ESC_SPAN_PIECES=$SP ESC_K3_ABLATE=$A timeout -k 10 240 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host \
        $( [ $A = 0 ] || echo --no-parity ) > $OUT/full_sp${SP}_a$A.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
    show $OUT/full_sp${SP}_a$A.json "full span_pieces=$SP ablate=$A"
  done
  ESC_SPAN_PIECES=$SP timeout -k 10 240 python3 bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_sp$SP.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
  show $OUT/shard8_sp$SP.json "shard8 span_pieces=$SP"
done
echo "[job] $(date) done"
