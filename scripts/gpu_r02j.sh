#!/bin/bash
# round parity subset, default bench, tail timings (DMC_TAIL_TIMING variant)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_j.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_j.log; tail -2 gpurun_out/pytest_j.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_j.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_j.json 2> gpurun_out/bench_j.err || { tail -20 gpurun_out/bench_j.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_j.json')); print('ms_per_step', d['ms_per_step'], d['value']/1e6, d['stages_ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
cp dmclock_amd/variants/tail.so dmclock_amd/libdmclock_gpu.so
DMC_DEBUG=1 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/tail.json 2> gpurun_out/tail.err || { tail -5 gpurun_out/tail.err; exit 1; }
grep "dmc tails" gpurun_out/tail.err | tail -3
