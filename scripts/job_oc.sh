#!/bin/bash
# K5 chunk-size variants (ESC_ORD_CHUNK builds): ordering parity tests, config-5 bench and
# kernel-trace stats per variant library.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_oc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in ${VARIANTS:-oc8 oc16}; do
    lib=""; [ "$v" != base ] && lib=$PWD/escalator_amd/libescalator_hip_$v.so
    echo "[job] $(date) $v tests"
    ESC_LIB_PATH=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        -k "order or sort or config5 or fixture" > $OUT/pytest_$v.log 2>&1 || { tail -30 $OUT/pytest_$v.log; exit 1; }
    tail -1 $OUT/pytest_$v.log
    ESC_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$v -o run \
        -- python3 bench.py --config 5 --steps 20 --warmup 5 > $OUT/bench5_$v.json 2> $OUT/kt_$v.log || exit 1
    find $OUT/kt_$v -name "*kernel_stats.csv" -exec mv {} $OUT/kernel_stats_$v.csv \;
    rm -rf $OUT/kt_$v
done
echo "[job] $(date) done"
