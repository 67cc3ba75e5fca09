#!/bin/bash
# single-op path: parity (new + KATs + facade + U1 + maintenance), latency
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_single_op.py tests/test_dynamic_info.py tests/test_maintenance.py tests/test_facade_cpp.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -s > gpurun_out/pytest_r02c.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_r02c.log; tail -3 gpurun_out/pytest_r02c.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_r02c.log | head -30; exit $rc; }
for n in 10000 100000; do
  timeout -k 10 300 tests/cpp/latency $n 2000 > gpurun_out/latency_$n.json || exit $?
  cat gpurun_out/latency_$n.json
done
timeout -k 10 300 tests/cpp/latency 1048576 2000 --no-facade > gpurun_out/latency_1048576.json || exit $?
cat gpurun_out/latency_1048576.json
