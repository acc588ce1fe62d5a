#!/bin/bash
# Round 4: K2 + tracker as node blocks of K1's grid (ESC_K1_NODE) — parity, then the
# shard-of-8 and full steps with and without, and the tracker-set reload.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04l}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -k "k2_placement" -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest_k2.log 2>&1 || { tail -60 $OUT/pytest_k2.log; exit 1; }
tail -1 $OUT/pytest_k2.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
show() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,2), round(d['roofline']['launch_ms']*1e3,2), {k: round(v*1e3,1) for k, v in (d.get('stage_ms') or {}).items()}, round(d['roofline']['frac'],3), d.get('parity'))"; }
for K in 1 0; do
  ESC_K1_NODE=$K timeout -k 10 300 python -u bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_k$K.json 2> $OUT/shard8_k$K.err || { tail -30 $OUT/shard8_k$K.err; exit 1; }
  show $OUT/shard8_k$K.json "shard8 k1node=$K"
  ESC_K1_NODE=$K timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host \
      > $OUT/full_k$K.json 2> $OUT/full_k$K.err || { tail -30 $OUT/full_k$K.err; exit 1; }
  show $OUT/full_k$K.json "full k1node=$K"
done
echo "[job] $(date) reload"
timeout -k 10 600 python -u scripts/bench_reload.py > $OUT/reload.json 2> $OUT/reload.err || { tail -30 $OUT/reload.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/reload.json')); print(json.dumps(d))"
echo "[job] $(date) done"
