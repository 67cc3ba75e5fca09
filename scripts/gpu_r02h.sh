#!/bin/bash
# fast-record rounds: the whole -m gpu suite, then the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_h.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_h.log; tail -3 gpurun_out/pytest_h.log
[ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/pytest_h.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { tail -20 gpurun_out/bench_h.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_h.json')); print('ms_per_step', d['ms_per_step'], d['value']/1e6, d['stages_ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['engine_counters'])"
