#!/bin/bash
# fused histogram: bench-shaped and full-size parity, the round parity subset, default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "bench_shaped" -s > gpurun_out/pytest_k1.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_k1.log; grep "hint_misses" gpurun_out/pytest_k1.log | sed 's/.*sample_retries/sample_retries/' | head -8; tail -2 gpurun_out/pytest_k1.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_k1.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || { tail -20 gpurun_out/bench_k.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_k.json')); print('ms_per_step', d['ms_per_step'], d['value']/1e6, d['stages_ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['engine_counters'])"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_k2.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_k2.log; tail -2 gpurun_out/pytest_k2.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_k2.log | head -30; exit $rc; }
