#!/bin/bash
# A/B on one box: early summary on / off, alternating; then a kernel trace of the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab_on_$i.json 2> gpurun_out/ab_on_$i.err || { tail -5 gpurun_out/ab_on_$i.err; exit 1; }
  DMC_NO_EARLY_SUMMARY=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab_off_$i.json 2> gpurun_out/ab_off_$i.err || { tail -5 gpurun_out/ab_off_$i.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/ab_on_$i.json')); b=json.load(open('gpurun_out/ab_off_$i.json')); print('early on', a['ms_per_step'], 'off', b['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ab_trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile > gpurun_out/ab_trace.json 2> gpurun_out/ab_trace.err
rc=$?; echo "trace exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ab_trace.err; exit $rc; }
python tools/steps_timeline.py gpurun_out/ab_trace/run_kernel_trace.csv 3 | tail -20
