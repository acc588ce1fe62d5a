#!/bin/bash
# Iteration job: GPU parity tests, K1 variant timings, a short bench under a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-it}
echo "[job] $(date) pytest -m gpu"
timeout -k 10 420 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1 && tail -1 gpurun_out/pytest_gpu_${TAG}.log &&
echo "[job] $(date) k1 variants" &&
VARIANTS=${VARIANTS:-0,1,3,4,5,6,7,8} timeout -k 10 400 python -u scripts/k1_variants.py > gpurun_out/k1_variants_${TAG}.json 2>&1 &&
cat gpurun_out/k1_variants_${TAG}.json &&
echo "[job] $(date) bench under kernel trace" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o run \
    -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err &&
cat gpurun_out/bench_${TAG}.json && cut -c1-160 gpurun_out/prof_${TAG}/run_kernel_stats.csv &&
echo "[job] $(date) done"
