#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own hard time limit; no
# tracing domains are combined with --pmc): the decision kernels on config 4, then the
# ordering kernels on config 5 (HBM bytes only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pmc}
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
CMD5="python3 bench.py --config 5 --steps 3 --warmup 1"
rocprofv3 -L > gpurun_out/counters_${TAG}.txt 2>&1 || true
run() {   # prefix, regex, command, name, counters...
    local pre=$1 rx=$2 cmd=$3 name=$4; shift 4
    echo "[pmc] $(date) $pre $name: $*"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$rx" \
        --output-format csv -d gpurun_out/${pre}_${TAG}_${name} -o run -- $cmd > gpurun_out/${pre}_${TAG}_${name}.log 2>&1
}
K="k_pod_reduce|k_step_tail|k_node_groups"
S="k_ord_fused|k_ord_count|k_ord_scatter"
run pmc "$K" "$CMD" fetch FETCH_SIZE &&
run pmc "$K" "$CMD" write WRITE_SIZE &&
run pmc "$K" "$CMD" sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD &&
run pmc "$K" "$CMD" lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS &&
run pmc "$K" "$CMD" occ SQ_WAVES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_LDS_ATOMIC SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE GRBM_COUNT &&
run pmc5 "$S" "$CMD5" fetch FETCH_SIZE &&
run pmc5 "$S" "$CMD5" write WRITE_SIZE &&
echo "[pmc] $(date) done"
