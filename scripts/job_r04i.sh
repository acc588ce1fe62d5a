#!/bin/bash
# Round 4: K2 + tracker inside K1 (ESC_K1_NODE) and the node groups + decide in the tail's
# fold blocks (ESC_TAIL_FUSED): parity suite, then shard-of-8 and full steps per layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -k "step_layouts" -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest_layouts.log 2>&1 || { tail -60 $OUT/pytest_layouts.log; exit 1; }
tail -1 $OUT/pytest_layouts.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
show() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,2), {k: round(v*1e3,1) for k, v in (d.get('stage_ms') or {}).items()}, round(d['roofline']['frac'],3), d.get('parity'))"; }
for L in "1 1" "1 0" "0 0"; do
  set -- $L
  ESC_K1_NODE=$1 ESC_TAIL_FUSED=$2 timeout -k 10 300 python -u bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_$1$2.json 2> $OUT/shard8_$1$2.err || { tail -30 $OUT/shard8_$1$2.err; exit 1; }
  show $OUT/shard8_$1$2.json "shard8 k1node=$1 fused=$2"
  ESC_K1_NODE=$1 ESC_TAIL_FUSED=$2 timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host \
      > $OUT/full_$1$2.json 2> $OUT/full_$1$2.err || { tail -30 $OUT/full_$1$2.err; exit 1; }
  show $OUT/full_$1$2.json "full k1node=$1 fused=$2"
done
for LIB in default exp/libescalator_rsu4.so; do
  if [ $LIB = default ]; then unset ESC_LIB_PATH; else export ESC_LIB_PATH=$PWD/escalator_amd/$LIB; fi
  timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5_$(basename $LIB).json 2> $OUT/bench5.err || { tail -30 $OUT/bench5.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench5_$(basename $LIB).json')); print('config5 $LIB', round(d['ms_per_step']*1e3,2), round(d['roofline']['frac'],3), d['age_index_build'], d['parity'])"
done
unset ESC_LIB_PATH
echo "[job] $(date) done"
