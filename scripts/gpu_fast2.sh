#!/bin/bash
# fast reservation+priority candidates: round parity subset, then A/B vs HEAD
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/f2_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/f2_pytest.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/f2_pytest.log | head -20; exit $rc; }
bash scripts/gpu_ab_run.sh
