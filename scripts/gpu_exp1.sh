#!/bin/bash
# timing experiments: stage times of the normal build, of emit without walks,
# and the last-block tail clocks
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
st() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ms_per_step', d['ms_per_step'], d['stages_ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])" "$@"; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e_base.json 2> gpurun_out/e_base.err || { tail -20 gpurun_out/e_base.err; exit 1; }
st gpurun_out/e_base.json base
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
cp dmclock_amd/variants/nowalk.so dmclock_amd/libdmclock_gpu.so
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/e_nowalk.json 2> gpurun_out/e_nowalk.err || { tail -20 gpurun_out/e_nowalk.err; exit 1; }
st gpurun_out/e_nowalk.json nowalk
cp dmclock_amd/variants/tail.so dmclock_amd/libdmclock_gpu.so
DMC_DEBUG=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/tail.json 2> gpurun_out/tail.err || { tail -20 gpurun_out/tail.err; exit 1; }
grep "dmc tails" gpurun_out/tail.err | tail -4
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
