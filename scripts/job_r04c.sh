#!/bin/bash
# Round 4 roofline evidence for the kernel that is timed: the bench line,
# then rocprofv3 --kernel-trace --stats of the SAME command, then separate --pmc passes
# (FETCH_SIZE, WRITE_SIZE; nothing else combined with --pmc), at full size (config 4, N=1)
# and at rank 0's shard of N=8 (--shard-of 8); scripts/prof_summary.py keeps the timed
# launches (K1: the 50 back-to-back launches bench.py times last) into gpurun_out/$TAG/profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04_prof}
OUT=gpurun_out/$TAG
PROF=$OUT/profiles          # copied into profiles/$TAG/ here afterwards (only gpurun_out/ returns)
mkdir -p $OUT $PROF
export TMPDIR=/tmp
K="k_pod_reduce|k_step_tail|k_node_groups|k_decide|k_ord_"
prof_set() {   # name, bench args...
    local name=$1; shift
    echo "[job] $(date) $name: bench"
    timeout -k 10 400 python3 -u bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -20 $OUT/bench_$name.err; return 1; }
    echo "[job] $(date) $name: kernel trace"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$name -o run \
        -- python3 bench.py "$@" > $OUT/trace_$name.log 2>&1 || { tail -20 $OUT/trace_$name.log; return 1; }
    echo "[job] $(date) $name: pmc fetch"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv \
        -d $OUT/fetch_$name -o run -- python3 bench.py "$@" --no-cpu-baseline --no-host > $OUT/fetch_$name.log 2>&1 || { tail -20 $OUT/fetch_$name.log; return 1; }
    echo "[job] $(date) $name: pmc write"
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv \
        -d $OUT/write_$name -o run -- python3 bench.py "$@" --no-cpu-baseline --no-host > $OUT/write_$name.log 2>&1 || { tail -20 $OUT/write_$name.log; return 1; }
    local tr=$(find $OUT/trace_$name -name "run_kernel_trace.csv" | head -1)
    local st=$(find $OUT/trace_$name -name "run_kernel_stats.csv" | head -1)
    local fe=$(find $OUT/fetch_$name -name "run_counter_collection.csv" | head -1)
    local wr=$(find $OUT/write_$name -name "run_counter_collection.csv" | head -1)
    cp $st $PROF/kernel_stats_$name.csv
    cp $OUT/bench_$name.json $PROF/bench_$name.json
    python3 scripts/prof_summary.py --trace $tr --fetch $fe --write $wr --last 50 --bench $OUT/bench_$name.json \
        --out $PROF/summary_$name.json
}
prof_set full --steps 20 --warmup 5 || exit 1
prof_set shard8 --shard-of 8 --steps 20 --warmup 5 || exit 1
# k_step_tail role ablations at rank 0's shard of N = 8 (timing only, wrong results:
# ESC_K3_ABLATE 8 no fold, 16 no node pieces, 32 no packed orderings)
for A in 0 8 16 32 48 56; do
    ESC_K3_ABLATE=$A timeout -k 10 240 python3 bench.py --shard-of 8 --steps 30 --warmup 5 > $OUT/tailabl_a$A.json 2> $OUT/tailabl.err ||
        { tail $OUT/tailabl.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/tailabl_a$A.json')); print('ablate $A', round(d['ms_per_step']*1e3, 1), {k: round(v*1e3, 1) for k, v in d['stage_ms'].items()})"
done
echo "[job] $(date) done"
