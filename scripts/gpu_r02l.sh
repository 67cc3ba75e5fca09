#!/bin/bash
# fused histogram diagnostics: debug bench rounds, then the 1M fused-call parity test
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
DMC_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 6 --warmup 2 > gpurun_out/l_dbg.json 2> gpurun_out/l_dbg.err
rc=$?; echo "debug bench exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/l_dbg.err; exit $rc; }
grep "dmc round" gpurun_out/l_dbg.err | tail -12 | sed 's/dmc round: //' | cut -c1-260
python -c "import json; d=json.load(open('gpurun_out/l_dbg.json')); print(d['engine_counters'])"
timeout -k 10 300 python -u -m pytest tests/test_device_parity.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "fused_bench_call" > gpurun_out/l_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/l_pytest.log
