#!/bin/bash
# N=2 rehearsal on one GPU (two ranks on device 0, gloo host-staged exchange): the
# multi-rank bench path end to end with rank-0 parity, config 4 at 12.5M pods per rank.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/${TAG:-n2}
mkdir -p $OUT
ESC_BENCH_BACKEND=gloo ESC_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --pods 25000000 --steps 5 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_n2_rehearsal.json 2> $OUT/n2.err || { tail -30 $OUT/n2.err; exit 1; }
cat $OUT/bench_n2_rehearsal.json
echo done
