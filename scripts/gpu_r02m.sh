#!/bin/bash
# fused histogram cost: default build (fused / not fused) and a 1-block-per-CU scan build
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/m_$1.json 2> gpurun_out/m_$1.err || { tail -5 gpurun_out/m_$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/m_$1.json')); print('$1', d['ms_per_step'], d['stages_ms_per_step'], d['engine_counters']['hint_misses'])"
}
run fused
DMC_NO_FUSE_HIST=1 run nofuse
cp dmclock_amd/variants/minw4.so dmclock_amd/libdmclock_gpu.so
run minw4
DMC_NO_FUSE_HIST=1 run minw4_nofuse
