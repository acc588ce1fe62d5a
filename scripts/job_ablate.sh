cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
VARIANTS=0,9,10,11,12,13 timeout -k 10 300 python -u scripts/k1_variants.py > gpurun_out/k1_ablate.json 2>&1 && cat gpurun_out/k1_ablate.json
