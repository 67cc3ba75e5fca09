#!/bin/bash
# fast-record rounds: round parity subset, default bench, a debug bench (candidate kinds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_i.log; tail -3 gpurun_out/pytest_i.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_i.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_i.json 2> gpurun_out/bench_i.err || { tail -20 gpurun_out/bench_i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_i.json')); print('ms_per_step', d['ms_per_step'], d['value']/1e6, d['stages_ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
DMC_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_idbg.json 2> gpurun_out/bench_idbg.err || { tail -20 gpurun_out/bench_idbg.err; exit 1; }
grep "dmc round" gpurun_out/bench_idbg.err | tail -3 | sed 's/.*pgroups/pgroups/'
