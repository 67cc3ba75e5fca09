#!/bin/bash
# config 5 A/B: variants/head.so (before the interleaved apply) vs cur.so
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
for round in 1 2; do
for v in head cur; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5ab_$v.json 2> gpurun_out/c5ab_$v.err || { tail -5 gpurun_out/c5ab_$v.err; cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5ab_$v.json')); print('$v', d['ms_per_step'], round(d['value']/1e6))"
done
done
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
