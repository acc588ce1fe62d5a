#!/bin/bash
# Config #5 orderings at N=1 and a 2-rank rehearsal (gloo, both ranks on the one device of
# this box), then the PMC passes of scripts/pmc_job.sh.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r01_v8}
echo "[job] $(date) config 5, N=1"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 3 > gpurun_out/bench5_${TAG}.json 2> gpurun_out/bench5_${TAG}.err &&
cat gpurun_out/bench5_${TAG}.json &&
echo "[job] $(date) config 5, 2-rank rehearsal" &&
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --config 5 --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/bench5_n2_${TAG}.json 2> gpurun_out/bench5_n2_${TAG}.err &&
cat gpurun_out/bench5_n2_${TAG}.json &&
echo "[job] $(date) pmc" &&
TAG=$TAG bash scripts/pmc_job.sh &&
echo "[job] $(date) done"
