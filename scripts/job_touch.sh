#!/bin/bash
# Compact K1 flush + pair0-bucket pod order: GPU suite under each ESC_POD_SORT setting
# (SUITE_SORTS), then config 4 + rank-0-of-8 benches per setting (SETTINGS: "name:ENV=V,ENV=V").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_touch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for srt in ${SUITE_SORTS:-0}; do
    echo "[job] $(date) pytest -m gpu (ESC_POD_SORT=$srt)"
    ESC_POD_SORT=$srt timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu_sort$srt.log 2>&1 || { tail -40 $OUT/pytest_gpu_sort$srt.log; exit 1; }
    tail -1 $OUT/pytest_gpu_sort$srt.log
done
for st in $SETTINGS; do
    name=${st%%:*}; envs=${st#*:}
    echo "[job] $(date) bench $name ($envs)"
    env ${envs//,/ } timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-host \
        > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail $OUT/bench_$name.err; exit 1; }
    env ${envs//,/ } timeout -k 10 240 python bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
        > $OUT/bench_shard8_$name.json 2> $OUT/bench_shard8_$name.err || { tail $OUT/bench_shard8_$name.err; exit 1; }
    python - $OUT/bench_$name.json $OUT/bench_shard8_$name.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f)); r = d["roofline"]
    print(f.split("/")[-1], "step %.4f ms  K1 %.4f ms frac %.3f" % (d["ms_per_step"], r["launch_ms"], r["frac"]),
          {k: round(v * 1e3, 1) for k, v in d["stage_ms"].items()}, d["parity"])
PY
done
echo "[job] $(date) done"
