#!/bin/bash
# Round 4: fused tail (node groups + decide inside k_step_tail) — parity suite, then the
# shard-of-8 and full-size step with and without the fusion.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu (relabel first)"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu -k "relabel or multi_device_events" \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "[job] $(date) bench shard-of-8 fused / unfused"
for F in 1 0; do
  ESC_TAIL_FUSED=$F timeout -k 10 300 python -u bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_f$F.json 2> $OUT/shard8_f$F.err || { tail -30 $OUT/shard8_f$F.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/shard8_f$F.json')); print('fused=$F', d['ms_per_step'], d.get('stage_ms'), d['roofline']['frac'])"
done
for F in 1 0; do
  ESC_TAIL_FUSED=$F timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host \
      > $OUT/full_f$F.json 2> $OUT/full_f$F.err || { tail -30 $OUT/full_f$F.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/full_f$F.json')); print('full fused=$F', d['ms_per_step'], d.get('stage_ms'), d['roofline']['frac'])"
done
echo "[job] $(date) smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo "[job] $(date) done"
