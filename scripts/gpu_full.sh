#!/bin/bash
# GPU-box run (round 1): tests, then bench, then rocprof kernel stats.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-profile --no-cpu-baseline > gpurun_out/bench_noprof.json 2> gpurun_out/bench_noprof.err
rc=$?; [ $rc -eq 0 ] || { echo "bench2 failed $rc"; tail -30 gpurun_out/bench_noprof.err; exit $rc; }
cat gpurun_out/bench_noprof.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; echo "rocprof exit $rc"; exit $rc
