#!/bin/bash
# Round 4: age-index scatter with whole-line digit runs (a build with -DESC_RS_CARRY=1 in
# escalator_amd/exp/; LIBS names other builds there) against the default: K5 parity, config-5 index build, scatter writes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for L in ${LIBS:-default carry}; do
  if [ $L != default ]; then export ESC_LIB_PATH=$PWD/escalator_amd/exp/libescalator_$L.so; else unset ESC_LIB_PATH; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu -k "sort or order or age or synthetic or node_index or relabel or nodes_add" \
      -x -v --timeout 200 --timeout-method thread > $OUT/pytest_k5_$L.log 2>&1 || { tail -60 $OUT/pytest_k5_$L.log; exit 1; }
  echo "$L: $(tail -1 $OUT/pytest_k5_$L.log)"
  timeout -k 10 300 python3 -u bench.py --config 5 --steps 20 --warmup 3 > $OUT/bench5_$L.json 2> $OUT/bench5.err || { tail -20 $OUT/bench5.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench5_$L.json')); print('$L config5', round(d['ms_per_step']*1e3,2), d['age_index_build'], d['parity'])"
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_rs_scatter" --output-format csv -d $OUT/wr_$L -o run \
      -- python3 bench.py --config 5 --steps 3 --warmup 1 > $OUT/wr_$L.log 2>&1 || { tail -20 $OUT/wr_$L.log; exit 1; }
  f=$(find $OUT/wr_$L -name run_counter_collection.csv | head -1)
  python3 - "$f" "$L" <<'PY'
import csv, sys, collections
per = collections.defaultdict(float)
name = {}
for r in csv.DictReader(open(sys.argv[1])):
    per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    name[r["Dispatch_Id"]] = "final" if "true" in r["Kernel_Name"].split("(")[0] else "pass"
agg = collections.defaultdict(list)
for d, v in per.items():
    agg[name[d]].append(v * 1024)
for k, v in agg.items():
    print(sys.argv[2], k, "launches", len(v), "mean write MB", round(sum(v) / len(v) / 1e6, 2))
PY
done
echo "[job] $(date) done"
