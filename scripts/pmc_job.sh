#!/bin/bash
# PMC passes for the dominant kernel (one counter group per rocprofv3 run, each under its
# own hard time limit; no tracing domains are combined with --pmc).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1 || true
run() {   # name, counters...
    local name=$1; shift
    echo "[pmc] $(date) $name: $*"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "k_pod_reduce|k_node_pieces|k_combine" \
        --output-format csv -d gpurun_out/pmc_${TAG}_${name} -o run -- $CMD > gpurun_out/pmc_${TAG}_${name}.log 2>&1
}
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run occ SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_LDS_ATOMIC SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE GRBM_COUNT &&
echo "[pmc] $(date) done"
