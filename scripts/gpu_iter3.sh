#!/bin/bash
# gpu_iter2.sh, then the DMC_TAIL_TIMING build's tail timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash scripts/gpu_iter2.sh || exit $?
cp dmclock_amd/variants/tail.so dmclock_amd/libdmclock_gpu.so
DMC_DEBUG=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_ARGS} > gpurun_out/tail.json 2> gpurun_out/tail.err
rc=$?; [ $rc -eq 0 ] || { echo "tail bench failed $rc"; tail -30 gpurun_out/tail.err; exit $rc; }
grep "dmc tails" gpurun_out/tail.err | tail -6
