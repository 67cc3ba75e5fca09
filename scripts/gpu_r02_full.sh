#!/bin/bash
# round-2 full check, as the driver runs it: the whole -m gpu suite, smoke(),
# the default bench command (with the CPU baseline)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_full.log; tail -3 gpurun_out/pytest_full.log
[ $rc -eq 0 ] || { grep -n "FAIL\|Error" gpurun_out/pytest_full.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_default.err; exit $rc; }
cat gpurun_out/bench_default.json
