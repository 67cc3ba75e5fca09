#!/bin/bash
# activation chain speculation: parity (churn/activation/config 4) + config-4 bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_single_op.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "churn or activation or config4 or single_op or undercut or chunks" > gpurun_out/pytest_r02f.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_r02f.log; tail -3 gpurun_out/pytest_r02f.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_r02f.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4.json')); print('ms_per_step', d['ms_per_step'], d['stages_ms_per_step'], d.get('activations_per_step'))"
DMC_DEBUG=1 timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --steps 2 --warmup 2 > gpurun_out/c4dbg.json 2> gpurun_out/c4dbg.err
grep act_resolve gpurun_out/c4dbg.err | tail -4
