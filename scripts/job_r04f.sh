#!/bin/bash
# Round 4: fused tail v2 (fold blocks last, batched column counts) — parity suite, shard-of-8
# and full step fused / unfused, then K1 loads-only ablations at shard size (plan vs per-wave
# shares: do class-run restarts cost the shard's K phase?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
show() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,2), {k: round(v*1e3,1) for k, v in (d.get('stage_ms') or {}).items()}, round(d['roofline']['frac'],3))"; }
for F in 1 0; do
  ESC_TAIL_FUSED=$F timeout -k 10 300 python -u bench.py --shard-of 8 --steps 200 --warmup 20 --no-cpu-baseline --no-host \
      > $OUT/shard8_f$F.json 2> $OUT/shard8_f$F.err || { tail -30 $OUT/shard8_f$F.err; exit 1; }
  show $OUT/shard8_f$F.json "shard8 fused=$F"
done
for F in 1 0; do
  ESC_TAIL_FUSED=$F timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host \
      > $OUT/full_f$F.json 2> $OUT/full_f$F.err || { tail -30 $OUT/full_f$F.err; exit 1; }
  show $OUT/full_f$F.json "full fused=$F"
done
echo "[job] $(date) config 5"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5.json 2> $OUT/bench5.err || { tail -30 $OUT/bench5.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench5.json')); print('config5', round(d['ms_per_step']*1e3,2), d['roofline'], d['age_index_build']['ms'], d['parity'])"
echo "[job] $(date) k1 trace at 12.5M pods (calibrated)"
PODS=12500000 CALIBRATE=10 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/k1_trace_p12.json 2> $OUT/k1_trace.err || { tail -30 $OUT/k1_trace.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/k1_trace_p12.json'))['variants']['0']; print({k: d[k] for k in ('kernel_us','k_phase_us_mean','k_phase_us_max','end_spread_us','k_phase_fit_us','runs_hist','k_phase_mean_by_runs')})"
echo "[job] $(date) done"
