#!/bin/bash
# Round 4: node groups load K4's inputs beside the piece rows — parity suite, then the
# config-4 step twice (node-groups stage) and its kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04u}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
show() { python3 -c "import json; d=json.load(open('$1')); print('$2', round(d['ms_per_step']*1e3,1), round(d['roofline']['launch_ms']*1e3,1), {k: round(v*1e3,1) for k, v in d['stage_ms'].items()}, d.get('parity'))"; }
for R in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host > $OUT/full_$R.json 2> $OUT/err.log || { tail $OUT/err.log; exit 1; }
  show $OUT/full_$R.json "full $R"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
    -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-host --no-parity > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
st=$(find $OUT/trace -name "run_kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.DictReader(open('$st')):
    n = r['Name'].split('(')[0].replace('void ', '').replace('esc::', '')
    if any(k in n for k in ('k_pod_reduce', 'k_step_tail', 'k_node_groups')):
        print(n[:40], r['Calls'], round(float(r['AverageNs'])/1000, 2))
"
echo "[job] $(date) done"
