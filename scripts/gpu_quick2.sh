#!/bin/bash
# quick check: GPU parity subset, bench, per-candidate apply timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_iter.log; tail -2 gpurun_out/pytest_iter.log
[ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/pytest_iter.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('ms_per_step', d['ms_per_step'], d['stages_ms_per_step'])"
bash scripts/gpu_atime.sh
