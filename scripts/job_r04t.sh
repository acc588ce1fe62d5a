#!/bin/bash
# Round 4 final evidence: GPU suite, smoke, the default bench line, config 5, then the
# roofline profiles of the final build (scripts/job_r04c.sh -> gpurun_out/r04_prof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04t}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print({k: d[k] for k in ('value','ms_per_step','roofline','frac_baseline_md','parity')}); print(d.get('cpu_baseline'))"
timeout -k 10 300 python3 -u bench.py --config 5 > $OUT/bench5.json 2> $OUT/bench5.err || { tail -20 $OUT/bench5.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench5.json')); print(d['ms_per_step'], d['roofline'], d['age_index_build']['ms'], d['parity'])"
# N = 2 rehearsal on the one GPU (bench.py spawns its two ranks itself; gloo, both on device 0)
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 500 python3 bench.py --gpus 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-host > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { tail -30 $OUT/bench_n2.err; exit 1; }
grep -o '"n_gpus": [0-9]*\|"parity": "[^"]*"\|"exchange": "[^"]*"' $OUT/bench_n2.json
bash scripts/job_r04c.sh
