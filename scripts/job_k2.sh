# K2 variants: parity under the atomic node pass, then bench stage times for both.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
ESC_K2_VARIANT=1 timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k2.log 2>&1 &&
tail -1 gpurun_out/pytest_k2.log &&
ESC_K2_VARIANT=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k2v0.json 2>gpurun_out/bench_k2v0.err &&
ESC_K2_VARIANT=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k2v1.json 2>gpurun_out/bench_k2v1.err &&
python3 -c "
import json
for v in (0, 1):
    d = json.load(open('gpurun_out/bench_k2v%d.json' % v))
    print(v, d['ms_per_step'], d['stage_ms'], d['parity'])
"
