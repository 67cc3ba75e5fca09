#!/bin/bash
# timing experiment: apply without the slow candidates' re-walks (wrong results)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
for v in head noslow head noslow; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/ns_$v.json 2> gpurun_out/ns_$v.err || { tail -3 gpurun_out/ns_$v.err; }
  python -c "import json; d=json.load(open('gpurun_out/ns_$v.json')); print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()})" || true
done
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
