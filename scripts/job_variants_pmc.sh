cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp &&
timeout -k 10 300 python -u scripts/k1_variants.py > gpurun_out/k1_variants_r01c.json 2>&1 && cat gpurun_out/k1_variants_r01c.json &&
TAG=r01c bash scripts/pmc_job.sh
