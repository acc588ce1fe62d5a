#!/bin/bash
# Round 4: reload bench (trackers set on the packer), K1 dynamic shares (variant 5) vs the
# static plan at a rank's shard and at config 4, and the K1 trace at the shard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04k}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) reload"
timeout -k 10 600 python -u scripts/bench_reload.py > $OUT/reload.json 2> $OUT/reload.err || { tail -30 $OUT/reload.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/reload.json')); d.pop('raw_s', None); print(json.dumps(d))"
show() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,2), round(d['roofline']['launch_ms']*1e3,2), {k: round(v*1e3,1) for k, v in (d.get('stage_ms') or {}).items()}, round(d['roofline']['frac'],3), d.get('parity'))"; }
for V in 0 5; do
  ESC_K1_VARIANT=$V timeout -k 10 300 python -u bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_v$V.json 2> $OUT/shard8_v$V.err || { tail -30 $OUT/shard8_v$V.err; exit 1; }
  show $OUT/shard8_v$V.json "shard8 k1 variant $V"
  ESC_K1_VARIANT=$V timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host \
      > $OUT/full_v$V.json 2> $OUT/full_v$V.err || { tail -30 $OUT/full_v$V.err; exit 1; }
  show $OUT/full_v$V.json "full k1 variant $V"
done
echo "[job] $(date) done"
