#!/bin/bash
# State of the secondary paths: K1 per-workgroup timeline at shard size, config 5 orderings,
# scale-down reaping, informer events.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_state}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) k1 trace 12.5M"
PODS=12500000 CALIBRATE=16 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/k1_trace_p12.json 2> $OUT/k1_trace.err || { tail $OUT/k1_trace.err; exit 1; }
python -c "
import json; d = json.load(open('$OUT/k1_trace_p12.json'))['variants']['0']
print({k: v for k, v in d.items() if not isinstance(v, (list, dict))})"
echo "[job] $(date) config 5"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; exit 1; }
cut -c1-1500 $OUT/bench5.json
echo "[job] $(date) reaping"
timeout -k 10 400 python -u scripts/bench_reaping.py --steps 20 --warmup 3 > $OUT/bench_reaping.json 2> $OUT/bench_reaping.err || { tail $OUT/bench_reaping.err; exit 1; }
cut -c1-1500 $OUT/bench_reaping.json
echo "[job] $(date) events"
timeout -k 10 400 python -u scripts/bench_events.py > $OUT/events.json 2> $OUT/events.err || { tail $OUT/events.err; exit 1; }
cut -c1-1500 $OUT/events.json
echo "[job] $(date) done"
