#!/bin/bash
# HBM bytes (FETCH_SIZE, WRITE_SIZE; one counter per rocprofv3 pass) of the decision kernels
# on rank 0's shard of an N=8 run (bench --shard-of 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmcshard}
CMD="python3 bench.py --shard-of 8 --steps 3 --warmup 1 --no-cpu-baseline"
K="k_pod_reduce|k_step_tail|k_node_groups"
for C in FETCH_SIZE WRITE_SIZE; do
    echo "[pmc] $(date) $C"
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$K" \
        --output-format csv -d gpurun_out/${TAG}_$C -o run -- $CMD > gpurun_out/${TAG}_$C.log 2>&1 || exit 1
done
echo "[pmc] $(date) done"
