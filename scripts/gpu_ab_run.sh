#!/bin/bash
# A/B on one box: dmclock_amd/variants/head.so vs variants/cur.so (built by
# scripts/ab_build.sh), alternating, 3 rounds.  The variants load through
# DMC_LIB: the shipped dmclock_amd/libdmclock_gpu.so is never overwritten.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for round in 1 2 3; do
for v in head cur; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -5 gpurun_out/ab_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()})"
done
done
