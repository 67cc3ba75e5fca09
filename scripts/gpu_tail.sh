#!/bin/bash
# Tail timing of the last-block kernels (DMC_TAIL_TIMING build) and the
# config-3 bench on the normal build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
cp dmclock_amd/variants/tail.so dmclock_amd/libdmclock_gpu.so
DMC_DEBUG=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-profile ${BENCH_ARGS} > gpurun_out/tail.json 2> gpurun_out/tail.err
rc=$?; [ $rc -eq 0 ] || { echo "tail bench failed $rc"; tail -30 gpurun_out/tail.err; exit $rc; }
grep "dmc tails" gpurun_out/tail.err | tail -8
