#!/bin/bash
# GPU-box: GPU suite, config-4 bench, kernel trace of config-4 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 2 ${BENCH_ARGS} > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench_c4.err; exit $rc; }
cat gpurun_out/bench_c4.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python3 $R/bench.py --config 4 --steps 4 --warmup 2 --no-cpu-baseline --no-profile > $R/gpurun_out/prof_c4_bench.json 2> $R/gpurun_out/prof_c4.err
rc=$?; echo "rocprof exit $rc"; exit $rc
