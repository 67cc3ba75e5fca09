#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_eclk.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_eclk.log; tail -2 gpurun_out/pytest_eclk.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_eclk.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('ms_per_step', d['ms_per_step'], d['stages_ms_per_step'])"
DMC_DEBUG=1 DMC_EMIT_CLOCKS=1 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/eclk.json 2> gpurun_out/eclk.err
grep "emit clock" gpurun_out/eclk.err | tail -5
