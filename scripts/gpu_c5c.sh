#!/bin/bash
# config 5: hardware queues per process 4 (default) vs 8 (one per server stream)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for hq in 4 8; do
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 500 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5c_$hq.json 2> gpurun_out/c5c_$hq.err
  rc=$?; echo "config5 hwq $hq exit $rc"; [ $rc -eq 0 ] || { tail -10 gpurun_out/c5c_$hq.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/c5c_$hq.json')); print('hwq $hq', d['ms_per_step'], d['value']/1e6)"
done
