#!/bin/bash
# A/B of the variants in $VARIANTS (scripts/gpu_variants.sh), then the -m gpu
# suite on the shipped library
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_variants.sh || exit 1
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/suite.log 2>&1
rc=$?; tail -3 gpurun_out/suite.log; exit $rc
