#!/bin/bash
# Decision-step overhead study: the bench step time with K2 forked / zero-copy decisions on/off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity"
for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    echo "[step] ESC_NO_FORK=$1 ESC_NO_ZEROCOPY=$2"
    ESC_NO_FORK=$1 ESC_NO_ZEROCOPY=$2 timeout -k 10 200 $B 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['launch_ms'], d['stage_ms'])" || exit 1
done
