#!/bin/bash
# K3 (k_fold_decide) ablations and row-block sizes at shard size (12.5M pods), stage timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
OUT=gpurun_out/k3
mkdir -p $OUT
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --pods 12500000 --steps 30 --warmup 10 --no-cpu-baseline --no-parity > $OUT/$name.json 2> $OUT/$name.err || exit 1
}
run base ESC_K3_ABLATE=0
run no_last ESC_K3_ABLATE=1
run no_fold ESC_K3_ABLATE=4
run no_both ESC_K3_ABLATE=5


run nozc ESC_NO_ZEROCOPY=1
echo done
