#!/bin/bash
# Round 4: the fused-tail parity tests (ESC_TAIL_FUSED=1 beside the default), then the
# roofline evidence of the default step (scripts/job_r04c.sh -> gpurun_out/r04_prof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
echo "[job] $(date) fused-tail tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_multi.py -m gpu \
    -k "tail_fused or tracker_updates or multi_device_context" -x -v --timeout 200 --timeout-method thread \
    > gpurun_out/r04h/pytest_fused.log 2>&1 || { tail -60 gpurun_out/r04h/pytest_fused.log; exit 1; }
tail -2 gpurun_out/r04h/pytest_fused.log
bash scripts/job_r04c.sh
