#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py tests/test_single_op.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_r02g.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_r02g.log; tail -3 gpurun_out/pytest_r02g.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_r02g.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('ms_per_step', d['ms_per_step'], d['stages_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
