#!/bin/bash
# Round 4: what the tail's K2 role waits on — SQ counters of k_step_tail at config 4 with
# every role (ESC_K3_ABLATE=0) and with K2 alone (40), one --pmc pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
for A in 0 40 48 24; do
  ESC_K3_ABLATE=$A timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "k_step_tail" --output-format csv \
      -d $OUT/pmc_a$A -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host --no-parity > $OUT/pmc_a$A.log 2>&1 || { tail -20 $OUT/pmc_a$A.log; exit 1; }
  f=$(find $OUT/pmc_a$A -name run_counter_collection.csv | head -1)
  python3 - "$f" "$A" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
per = collections.defaultdict(list)
for r in rows:
    per[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("ablate", sys.argv[2], {k: round(sum(v[-10:]) / len(v[-10:])) for k, v in sorted(per.items())})
PY
done
echo "[job] $(date) done"
