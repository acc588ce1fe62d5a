#!/bin/bash
# k_memb_keys ablations (config 5 index build): kernel-trace stats per variant library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_mk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-base mk1 mk2 mk3}; do
    lib=""; [ "$v" != base ] && lib=$PWD/escalator_amd/libescalator_hip_$v.so
    echo "[job] $(date) $v"
    ESC_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o run \
        -- python3 bench.py --config 5 --steps 5 --warmup 2 > $OUT/kt_$v.log 2>&1 || exit 1
    find $OUT/kt_$v -name "*kernel_stats.csv" -exec mv {} $OUT/kernel_stats_$v.csv \;
    rm -rf $OUT/kt_$v
done
echo "[job] $(date) done"
