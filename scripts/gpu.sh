#!/bin/bash
# The GPU recipes in one place (run through gpurun from the repo root; every GPU step has
# its own time limit and the first failure ends the job).  Stages, in the order given:
#   suite            pytest -m gpu (-x), then __graft_entry__.smoke()
#   bench            the default bench line (config 4, N = 1), rank 0 of N = 8 (--shard-of 8),
#                    config 5 (orderings + age index)
#   ablate:NAME:A,.. the tail without some of its roles (measurement library, ESC_K3_ABLATE=A;
#                    timing only: wrong results) for profile NAME's bench command
#   nosel            config 4 and rank 0 of 8 without selections (--no-select)
#   rehearse2        N = 2 on one device: two gloo ranks (bench.py --gpus 2, ESC_BENCH_BACKEND=gloo,
#                    ESC_BENCH_DEVICE=0), and one process driving two shards (peer exchange)
#   rehearse2c5      config 5 (10 M nodes) at N = 2 on one device: two gloo ranks, each ordering its
#                    half of the nodes, the merged selections checked against the oracle
#   prof:NAME        rocprofv3 --kernel-trace --stats, then separate --pmc FETCH_SIZE and --pmc
#                    WRITE_SIZE passes of the same bench command, reduced by scripts/prof_summary.py
#                    to $OUT/profiles/summary_NAME.json.  NAME: full (config 4), shard8, config5
#   rt:NAME          rocprofv3 --kernel-trace --memory-copy-trace of the bench command (6 steps)
#   pmcsq:NAME       SQ counter pass (one --pmc run) of the same command
#   py:SCRIPT        python3 scripts/SCRIPT (e.g. k1_trace.py), output to $OUT
#   variants:A,B,..  A/B timing of library builds (scripts/build_variant.sh NAME ...:
#                    escalator_amd/libescalator_hip_NAME.so; "base" = the product library):
#                    rank 0 of 8 and config 4, each in turn, twice
#   variants5:A,B,.. the same for config 5 (age-index build and ordering times)
# usage: TAG=r05a scripts/gpu.sh suite bench prof:shard8
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
PROF=$OUT/profiles
mkdir -p $OUT $PROF
export TMPDIR=/tmp
STEPS=${STEPS:-20}

args_of() {    # the bench command of a profile name
    case $1 in
        full) echo "--steps $STEPS --warmup 5" ;;
        shard8) echo "--shard-of 8 --steps $STEPS --warmup 5" ;;
        config5) echo "--config 5 --steps $STEPS --warmup 3" ;;
        *) echo "unknown profile $1" >&2; return 1 ;;
    esac
}
last_of() {    # launches prof_summary keeps: K1's 50 timed launches, or config 5's cold steps + 1
    case $1 in config5) echo $((STEPS + 1)) ;; *) echo 50 ;; esac
}

suite() {
    echo "[gpu] $(date +%T) pytest -m gpu"
    timeout -k 10 1500 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread \
        > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; return 1; }
    tail -2 $OUT/pytest_gpu.log
    echo "[gpu] $(date +%T) smoke"
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; return 1; }
}

bench() {
    echo "[gpu] $(date +%T) bench config 4"
    timeout -k 10 500 python3 -u bench.py --steps $STEPS --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; return 1; }
    cut -c1-900 $OUT/bench.json
    echo "[gpu] $(date +%T) bench rank 0 of 8"
    timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
        > $OUT/bench_shard8.json 2> $OUT/bench_shard8.err || { tail $OUT/bench_shard8.err; return 1; }
    cut -c1-900 $OUT/bench_shard8.json
    echo "[gpu] $(date +%T) bench config 5"
    timeout -k 10 400 python3 -u bench.py --config 5 --steps $STEPS --warmup 3 > $OUT/bench5.json 2> $OUT/bench5.err || { tail $OUT/bench5.err; return 1; }
    cat $OUT/bench5.json
}

nosel() {      # the bench without selections (esc_set_selections off): their cost in the step
    echo "[gpu] $(date +%T) bench without selections: config 4, rank 0 of 8"
    timeout -k 10 400 python3 -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-host --no-select \
        > $OUT/bench_nosel.json 2> $OUT/bench_nosel.err || { tail $OUT/bench_nosel.err; return 1; }
    timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline --no-host --no-select \
        > $OUT/bench_shard8_nosel.json 2> $OUT/bench_shard8_nosel.err || { tail $OUT/bench_shard8_nosel.err; return 1; }
    python3 -c "
import json
for n in ('bench_nosel', 'bench_shard8_nosel'):
    d = json.load(open('$OUT/%s.json' % n))
    print(' ', n, 'step %.4f ms' % d['ms_per_step'], {k: round(x * 1e3, 1) for k, x in (d.get('stage_ms') or {}).items()})"
}

ablate() {     # NAME:A,B,..  the tail's roles dropped (measurement library, ESC_K3_ABLATE; wrong results)
    local name=${1%%:*} list=${1#*:} a args
    args=$(args_of $name) || return 1
    for a in ${list//,/ }; do
        echo "[gpu] $(date +%T) ablate $name $a"
        ESC_LIB_PATH=$PWD/escalator_amd/libescalator_hip_measure.so ESC_K3_ABLATE=$a timeout -k 10 300 python3 -u bench.py \
            $args --no-cpu-baseline --no-host --no-parity > $OUT/abl_${name}_$a.json 2> $OUT/abl_${name}_$a.err \
            || { tail $OUT/abl_${name}_$a.err; return 1; }
        python3 -c "
import json
d = json.load(open('$OUT/abl_${name}_$a.json'))
print('  $name a=$a step %.4f ms' % d['ms_per_step'], {k: round(x * 1e3, 1) for k, x in (d.get('stage_ms') or {}).items()})"
    done
}

rehearse2() {
    echo "[gpu] $(date +%T) N = 2 rehearsal: two gloo ranks on device 0"
    ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 10 --warmup 3 \
        --no-cpu-baseline > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail -30 $OUT/bench_n2_gloo.err; return 1; }
    cut -c1-900 $OUT/bench_n2_gloo.json
    echo "[gpu] $(date +%T) N = 2 rehearsal: one process, two shards on device 0 (peer exchange)"
    ESC_BENCH_DEVICES=0,0 timeout -k 10 600 python3 -u bench.py --gpus 2 --single-process --steps 10 --warmup 3 \
        --no-cpu-baseline > $OUT/bench_n2_multi.json 2> $OUT/bench_n2_multi.err || { tail -30 $OUT/bench_n2_multi.err; return 1; }
    cut -c1-900 $OUT/bench_n2_multi.json
}

rehearse2c5() {
    echo "[gpu] $(date +%T) N = 2 rehearsal of config 5: two gloo ranks on device 0"
    ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --config 5 --gpus 2 --steps 10 \
        --warmup 3 > $OUT/bench5_n2_gloo.json 2> $OUT/bench5_n2_gloo.err || { tail -30 $OUT/bench5_n2_gloo.err; return 1; }
    cut -c1-900 $OUT/bench5_n2_gloo.json
}

prof() {       # name
    local name=$1 a
    a=$(args_of $name) || return 1
    echo "[gpu] $(date +%T) prof $name: bench"
    timeout -k 10 500 python3 -u bench.py $a > $OUT/pbench_$name.json 2> $OUT/pbench_$name.err || { tail -20 $OUT/pbench_$name.err; return 1; }
    echo "[gpu] $(date +%T) prof $name: kernel trace"
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$name -o run \
        -- python3 bench.py $a --no-cpu-baseline --no-host > $OUT/trace_$name.log 2>&1 || { tail -20 $OUT/trace_$name.log; return 1; }
    echo "[gpu] $(date +%T) prof $name: pmc FETCH_SIZE"
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "(^|[ :])k_" --output-format csv -d $OUT/fetch_$name -o run \
        -- python3 bench.py $a --no-cpu-baseline --no-host > $OUT/fetch_$name.log 2>&1 || { tail -20 $OUT/fetch_$name.log; return 1; }
    echo "[gpu] $(date +%T) prof $name: pmc WRITE_SIZE"
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "(^|[ :])k_" --output-format csv -d $OUT/write_$name -o run \
        -- python3 bench.py $a --no-cpu-baseline --no-host > $OUT/write_$name.log 2>&1 || { tail -20 $OUT/write_$name.log; return 1; }
    local tr st fe wr
    tr=$(find $OUT/trace_$name -name "run_kernel_trace.csv" | head -1)
    st=$(find $OUT/trace_$name -name "run_kernel_stats.csv" | head -1)
    fe=$(find $OUT/fetch_$name -name "run_counter_collection.csv" | head -1)
    wr=$(find $OUT/write_$name -name "run_counter_collection.csv" | head -1)
    mkdir -p $PROF/raw_$name
    cp $st $PROF/kernel_stats_$name.csv
    # the profile's own bench line under its own name (the bench stage writes bench_*.json
    # in $OUT: a later stage can never overwrite what the summary was computed from)
    cp $OUT/pbench_$name.json $PROF/pbench_$name.json
    # the raw CSVs, cut to our kernels' columns, so the summary can be recomputed from the tree
    python3 - "$tr" "$fe" "$wr" "$PROF/raw_$name" <<'PY'
import csv, sys
tr, fe, wr, out = sys.argv[1:]
for src, dst, cols in ((tr, "kernel_trace.csv", ["Kernel_Name", "Dispatch_Id", "Start_Timestamp", "End_Timestamp"]),
                       (fe, "pmc_fetch.csv", ["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"]),
                       (wr, "pmc_write.csv", ["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])):
    with open(src) as f, open(out + "/" + dst, "w", newline="") as g:
        w = csv.writer(g)
        w.writerow(cols)
        for r in csv.DictReader(f):
            if r["Kernel_Name"].replace("void ", "").replace("esc::", "").startswith("k_"):
                w.writerow([r[c] for c in cols])
PY
    python3 scripts/prof_summary.py --trace $PROF/raw_$name/kernel_trace.csv --fetch $PROF/raw_$name/pmc_fetch.csv \
        --write $PROF/raw_$name/pmc_write.csv --last $(last_of $name) --bench $PROF/pbench_$name.json \
        --out $PROF/summary_$name.json
}

rt() {         # name: rocprofv3 --runtime-trace (HIP API + kernels + copies; no counters) of the bench command
    local name=$1 a
    a=$(args_of $name) || return 1
    echo "[gpu] $(date +%T) runtime trace $name"
    timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/rt_$name -o run \
        -- python3 bench.py $a --no-cpu-baseline --no-host > $OUT/rt_$name.log 2>&1 || { tail -20 $OUT/rt_$name.log; return 1; }
}

pmcsq() {      # name: one SQ counter pass (<= 8 SQ counters)
    local name=$1 a
    a=$(args_of $name) || return 1
    echo "[gpu] $(date +%T) pmc SQ $name"
    timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU \
        SQ_INSTS_LDS SQ_INSTS_VMEM_RD --kernel-include-regex "(^|[ :])k_" --output-format csv -d $OUT/sq_$name -o run \
        -- python3 bench.py $a --no-cpu-baseline --no-host > $OUT/sq_$name.log 2>&1 || { tail -20 $OUT/sq_$name.log; return 1; }
    find $OUT/sq_$name -name "run_counter_collection.csv" -exec cp {} $PROF/pmc_sq_$name.csv \;
}

variants() {   # comma-separated names
    local v lib
    for rep in 1 2; do
        for v in ${1//,/ }; do
            lib=$PWD/escalator_amd/libescalator_hip_$v.so
            [ "$v" = base ] && lib=$PWD/escalator_amd/libescalator_hip.so
            echo "[gpu] $(date +%T) variant $v (rep $rep)"
            ESC_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --shard-of 8 --steps 50 --warmup 10 --no-cpu-baseline \
                > $OUT/var_${v}_shard8_$rep.json 2> $OUT/var_${v}_shard8_$rep.err || { tail $OUT/var_${v}_shard8_$rep.err; return 1; }
            ESC_LIB_PATH=$lib timeout -k 10 400 python3 -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --no-host \
                --no-parity > $OUT/var_${v}_full_$rep.json 2> $OUT/var_${v}_full_$rep.err || { tail $OUT/var_${v}_full_$rep.err; return 1; }
            python3 -c "
import json
for n in ('shard8', 'full'):
    d = json.load(open('$OUT/var_${v}_%s_$rep.json' % n))
    print('  $v', n, 'step %.4f ms' % d['ms_per_step'], 'K1 %.4f ms' % d['roofline']['launch_ms'],
          {k: round(x * 1e3, 1) for k, x in (d.get('stage_ms') or {}).items()})"
        done
    done
}

variants5() {  # config 5 (age-index build, orderings) per library build
    local v lib
    for rep in 1 2; do
        for v in ${1//,/ }; do
            lib=$PWD/escalator_amd/libescalator_hip_$v.so
            [ "$v" = base ] && lib=$PWD/escalator_amd/libescalator_hip.so
            echo "[gpu] $(date +%T) variant $v config 5 (rep $rep)"
            ESC_LIB_PATH=$lib timeout -k 10 400 python3 -u bench.py --config 5 --steps $STEPS --warmup 3 --no-cpu-baseline \
                > $OUT/var5_${v}_$rep.json 2> $OUT/var5_${v}_$rep.err || { tail $OUT/var5_${v}_$rep.err; return 1; }
            python3 -c "
import json
d = json.load(open('$OUT/var5_${v}_$rep.json'))
print('  $v', 'index %.4f ms' % d['age_index_build']['ms'], 'order %.4f ms' % d['ms_per_step'])"
        done
    done
}

for stage in "$@"; do
    case $stage in
        suite) suite || exit 1 ;;
        bench) bench || exit 1 ;;
        rehearse2) rehearse2 || exit 1 ;;
        nosel) nosel || exit 1 ;;
        ablate:*) ablate ${stage#ablate:} || exit 1 ;;
        rehearse2c5) rehearse2c5 || exit 1 ;;
        prof:*) prof ${stage#prof:} || exit 1 ;;
        pmcsq:*) pmcsq ${stage#pmcsq:} || exit 1 ;;
        rt:*) STEPS=6 rt ${stage#rt:} || exit 1 ;;
        variants:*) variants ${stage#variants:} || exit 1 ;;
        variants5:*) variants5 ${stage#variants5:} || exit 1 ;;
        py:*) timeout -k 10 600 python3 -u scripts/${stage#py:} > $OUT/${stage#py:}.out 2>&1 || { tail -20 $OUT/${stage#py:}.out; exit 1; } ;;
        *) echo "unknown stage $stage"; exit 2 ;;
    esac
done
echo "[gpu] $(date +%T) done"
