#!/bin/bash
# Round 4: what k_decide's 9 us is — zero-copy decision stores to pinned host memory vs
# device memory (ESC_NO_ZEROCOPY=1), kernel trace of the shard-of-8 step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04m}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for Z in 0 1; do
  ESC_NO_ZEROCOPY=$Z timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_z$Z -o run \
      -- python3 bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline --no-host > $OUT/trace_z$Z.log 2>&1 || { tail -20 $OUT/trace_z$Z.log; exit 1; }
  st=$(find $OUT/trace_z$Z -name "run_kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$st')):
    n = r['Name'].split('(')[0].replace('void ', '').replace('esc::', '')
    if any(k in n for k in ('k_pod_reduce', 'k_step_tail', 'k_node_groups', 'k_decide', 'copyBuffer')):
        print('zerocopy-off=$Z', n[:40], r['Calls'], round(float(r['AverageNs'])/1000, 2))
"
  tail -1 $OUT/trace_z$Z.log | head -c 300; echo
done
echo "[job] $(date) done"
