#!/bin/bash
# K1 access-shape probe at shard and full size + K1 per-wave-share variants (needs ABLATIONS=1 build).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/shape
timeout -k 10 60 ./scripts/k1_shape_probe 12500000 > gpurun_out/shape/probe_p12.5M.json || exit 1
timeout -k 10 90 ./scripts/k1_shape_probe 100000000 > gpurun_out/shape/probe_p100M.json || exit 1
PODS=12500000 VARIANTS=0,6,12,14 ROUNDS=5 timeout -k 10 200 python -u scripts/k1_variants.py > gpurun_out/shape/k1ws_p12.5M.json 2> gpurun_out/shape/k1ws_p12.5M.err || exit 1
echo done
