#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
cp dmclock_amd/variants/norec.so dmclock_amd/libdmclock_gpu.so
DMC_DEBUG=1 DMC_EMIT_CLOCKS=1 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/e2.json 2> gpurun_out/e2.err
rc=$?
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
[ $rc -eq 0 ] || { tail -5 gpurun_out/e2.err; exit $rc; }
grep "emit c" gpurun_out/e2.err | tail -7
