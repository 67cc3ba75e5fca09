#!/bin/bash
# GPU-box: activation parity tests, then the config-4 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "activation or churn" > gpurun_out/pytest_act.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_act.log; tail -3 gpurun_out/pytest_act.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench_c4.err; exit $rc; }
cat gpurun_out/bench_c4.json
