#!/bin/bash
# Round 4: age-index scatter carrying each digit run's partial last line to the next chunk —
# K5 parity (then the suite), config 5 bench (index build ms), and WRITE_SIZE of the scatter.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu -k "sort or order or age or synthetic or node_index" \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest_k5.log 2>&1 || { tail -60 $OUT/pytest_k5.log; exit 1; }
tail -1 $OUT/pytest_k5.log
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for R in 1 2; do
  timeout -k 10 300 python3 -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5_$R.json 2> $OUT/bench5.err || { tail -20 $OUT/bench5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench5_$R.json')); print('config5', round(d['ms_per_step']*1e3,2), d['age_index_build'], d['parity'])"
done
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rs_scatter" --output-format csv -d $OUT/wr -o run \
    -- python3 bench.py --config 5 --steps 3 --warmup 1 > $OUT/wr.log 2>&1 || { tail -20 $OUT/wr.log; exit 1; }
f=$(find $OUT/wr -name run_counter_collection.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
per = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    per[(r["Kernel_Name"].split("(")[0][-40:], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
agg = collections.defaultdict(list)
for (k, _), v in per.items():
    agg[k].append(sum(v) * 1024)
for k, v in agg.items():
    print(k, "launches", len(v), "mean write MB", round(sum(v) / len(v) / 1e6, 2))
PY
echo "[job] $(date) done"
