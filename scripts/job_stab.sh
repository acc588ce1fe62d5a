#!/bin/bash
# Per-workgroup K1 duration stability across decisions (static shares), two sizes, in two
# separate processes (a fresh allocation each) to see whether the slow workgroups persist.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/stab
mkdir -p $OUT
for r in 1 2; do
PODS=100000000 VARIANTS=0 timeout -k 10 300 python -u scripts/k1_trace.py > $OUT/trace_p100M_$r.json 2> $OUT/t100.err || { tail $OUT/t100.err; exit 1; }
PODS=12500000 VARIANTS=0 timeout -k 10 200 python -u scripts/k1_trace.py > $OUT/trace_p12.5M_$r.json 2> $OUT/t12.err || { tail $OUT/t12.err; exit 1; }
done
echo done
