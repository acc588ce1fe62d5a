#!/bin/bash
# K1 per-wave shares (variant 6 / loads-only 14) against the per-workgroup default (0 / 12).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/k1ws
PODS=12500000 VARIANTS=0,6,12,14 ROUNDS=5 timeout -k 10 200 python scripts/k1_variants.py > gpurun_out/k1ws/p12.5M.json 2> gpurun_out/k1ws/p12.5M.err || exit 1
PODS=100000000 VARIANTS=0,6 ROUNDS=3 timeout -k 10 300 python scripts/k1_variants.py > gpurun_out/k1ws/p100M.json 2> gpurun_out/k1ws/p100M.err || exit 1
echo done
