# Quick GPU check: parity tests + K1 variant timings.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && TAG=${TAG:-q} &&
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 &&
tail -2 gpurun_out/pytest_gpu_${TAG}.log &&
VARIANTS=${VARIANTS:-0,9,10,11} timeout -k 10 300 python -u scripts/k1_variants.py > gpurun_out/k1_${TAG}.json 2>&1 && cat gpurun_out/k1_${TAG}.json
