#!/bin/bash
# Round 4: GPU suite, events bench (relabels/s), reload bench (parallel packer + load), then
# the roofline evidence (scripts/job_r04c.sh -> gpurun_out/r04_prof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "[job] $(date) events"
timeout -k 10 600 python -u scripts/bench_events.py > $OUT/events.json 2> $OUT/events.err || { tail -30 $OUT/events.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/events.json')); d.pop('raw_s', None); print(json.dumps(d))"
echo "[job] $(date) reload"
timeout -k 10 600 python -u scripts/bench_reload.py > $OUT/reload.json 2> $OUT/reload.err || { tail -30 $OUT/reload.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/reload.json')); d.pop('raw_s', None); print(json.dumps(d))"
bash scripts/job_r04c.sh
