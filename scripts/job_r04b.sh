#!/bin/bash
# Round 4: the whole GPU suite (node relabels, list drop-ins, two-process exchange, ...),
# smoke, and the events bench with relabels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu (new tests first)"
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu -k "relabel or multi_device_events" \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -60 $OUT/pytest_new.log; exit 1; }
tail -2 $OUT/pytest_new.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
echo "[job] $(date) smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log | tail -1
echo "[job] $(date) events"
timeout -k 10 600 python -u scripts/bench_events.py > $OUT/events.json 2> $OUT/events.err || { tail -30 $OUT/events.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/events.json')); d.pop('raw_s'); print(json.dumps(d))"
echo "[job] $(date) reload"
timeout -k 10 600 python -u scripts/bench_reload.py > $OUT/reload.json 2> $OUT/reload.err || { tail -30 $OUT/reload.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/reload.json')); d.pop('raw_s'); print(json.dumps(d))"
echo "[job] $(date) done"
