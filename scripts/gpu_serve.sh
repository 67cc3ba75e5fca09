#!/bin/bash
# the serve path (DMC_OPT_SERVE): single-op parity against the oracle, the
# facade KATs on it, then single-call latency at 1M clients (phase stamps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_single_op.py tests/test_facade_cpp.py > gpurun_out/serve_tests.log 2>&1
rc=$?; tail -3 gpurun_out/serve_tests.log; [ $rc = 0 ] || exit $rc
bash scripts/gpu_serve_lat.sh
