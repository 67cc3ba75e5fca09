#!/bin/bash
# A/B of the apply launch bound (variants base / mb2), then the GPU suite on the built library
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
VARIANTS="base mb2" bash scripts/gpu_variants_ab.sh || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/l_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/l_pytest.log; exit $rc
