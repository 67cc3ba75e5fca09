#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_single_op.py tests/test_gpu_parity.py tests/test_facade_cpp.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02d.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_r02d.log; tail -3 gpurun_out/pytest_r02d.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_r02d.log | head -30; exit $rc; }
bash scripts/gpu_lat_prof.sh
