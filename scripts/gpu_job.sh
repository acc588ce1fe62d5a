#!/bin/bash
# GPU validation + measurement job (run through gpurun).  Every GPU step has its own time
# limit and the steps are chained: the first failure ends the job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
echo "[job] $(date) pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 && echo "[job] pytest ok" &&
echo "[job] $(date) smoke" &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 &&
echo "[job] $(date) bench" &&
VARIANTS=${VARIANTS:-0,2,9,11,12,10} timeout -k 10 300 python -u scripts/k1_variants.py > gpurun_out/k1_variants_${TAG}.json 2>&1 && cat gpurun_out/k1_variants_${TAG}.json &&
timeout -k 10 400 python -u bench.py --steps ${STEPS} --warmup 5 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
cat gpurun_out/bench_${TAG}.json &&
echo "[job] $(date) config 5 orderings" &&
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/bench5_${TAG}.json 2> gpurun_out/bench5_${TAG}.err &&
cat gpurun_out/bench5_${TAG}.json &&
echo "[job] $(date) stream probe" &&
hipcc --offload-arch=gfx950 -O3 -o /tmp/stream_probe scripts/stream_probe.hip &&
timeout -k 10 120 /tmp/stream_probe > gpurun_out/stream_probe_${TAG}.json && cat gpurun_out/stream_probe_${TAG}.json &&
echo "[job] $(date) rocprofv3 kernel trace" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
    -- python3 bench.py --steps ${STEPS} --warmup 5 --no-cpu-baseline --no-parity \
    > gpurun_out/prof_${TAG}.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5_${TAG} -o run \
    -- python3 bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/prof5_${TAG}.log 2>&1 &&
echo "[job] $(date) done"
