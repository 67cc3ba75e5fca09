#!/bin/bash
# GPU-box: GPU suite, then the host-buffer API bench (PCIe inclusive).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --host-api --steps 20 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench_host.err; exit $rc; }
cat gpurun_out/bench_host.json
