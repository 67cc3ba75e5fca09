#!/bin/bash
# scan variants A/B on one box: HEAD, pre-issued R steps (2 slots, spills), 1 slot per
# thread, 2 slots at one block per CU; scan stage time and step time
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for round in 1 2; do
for v in head cur scan1 scan2w4; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sab_$v.json 2> gpurun_out/sab_$v.err || { tail -5 gpurun_out/sab_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sab_$v.json')); print('$v', d['ms_per_step'], 'scan', d['stages_ms_per_step']['scan'], 'emit', d['stages_ms_per_step']['emit'])"
done
done
cp dmclock_amd/variants/cur.so dmclock_amd/libdmclock_gpu.so
