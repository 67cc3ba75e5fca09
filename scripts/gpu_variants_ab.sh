#!/bin/bash
# A/B of the libraries in dmclock_amd/variants (VARIANTS="a b c"), alternating, 2 rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
for round in 1 2; do
for v in $VARIANTS; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/vab_$v.json 2> gpurun_out/vab_$v.err || { tail -5 gpurun_out/vab_$v.err; cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/vab_$v.json')); print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()}, d['engine_counters']['sample_retries'], d['engine_counters']['candidates'])"
done
done
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
