#!/bin/bash
# Round 4, first check: the new multi-process GPU tests (library words over gloo, 2 ranks on
# device 0), the reaping tests (ADVICE r3 upsert fix), and bench.py --gpus 2 without a
# launcher (it starts its own 2 ranks; gloo + one device: a rehearsal of the N = 2 shape).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu.py tests/test_harness.py -m gpu -k "dist or two_process or reaping or dropin or fixture_pods or fixture_nodes or harness" \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
echo "[job] $(date) bench --gpus 2 (self-launched, gloo, device 0)"
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 500 python bench.py --gpus 2 --steps 5 --warmup 2 \
    --no-cpu-baseline --no-host > $OUT/bench_n2.json 2> $OUT/bench_n2.err || { tail -30 $OUT/bench_n2.err; exit 1; }
cut -c1-400 $OUT/bench_n2.json
grep -o '"parity": "[^"]*"' $OUT/bench_n2.json
grep -o '"n_gpus": [0-9]*' $OUT/bench_n2.json
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 300 python bench.py --config 5 --gpus 2 --steps 5 --warmup 2 \
    > $OUT/bench5_n2.json 2> $OUT/bench5_n2.err || { tail -30 $OUT/bench5_n2.err; exit 1; }
cut -c1-300 $OUT/bench5_n2.json
grep -o '"parity": "[^"]*"' $OUT/bench5_n2.json
echo "[job] $(date) bench (N=1, full line)"
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['ms_per_step'], d['roofline']['frac'], d['parity']); print(json.dumps(d['host_side']))"
echo "[job] $(date) done"
