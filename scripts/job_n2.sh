#!/bin/bash
# N = 2 rehearsals on one GPU: two processes over gloo (host-staged exchange of the library's
# words, both ranks on device 0) and one process driving two shards of device 0
# (esc_ctx_create_multi's peer exchange); both check rank 0's decisions against the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03_n2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[job] $(date) torchrun 2 ranks (gloo, one device)"
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --no-host \
    > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { tail $OUT/bench_n2_gloo.err; exit 1; }
grep metric $OUT/bench_n2_gloo.json | cut -c1-300
grep -o '"parity": "[^"]*"' $OUT/bench_n2_gloo.json
echo "[job] $(date) single process, two shards of device 0"
ESC_BENCH_DEVICES=0,0 timeout -k 10 400 python bench.py --gpus 2 --single-process --steps 5 --warmup 2 --no-cpu-baseline \
    --no-host > $OUT/bench_n2_multi.json 2> $OUT/bench_n2_multi.err || { tail $OUT/bench_n2_multi.err; exit 1; }
grep -o '"parity": "[^"]*"' $OUT/bench_n2_multi.json
grep -o '"ms_per_step": [0-9.]*' $OUT/bench_n2_multi.json
echo "[job] $(date) done"
