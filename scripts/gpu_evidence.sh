#!/bin/bash
# GPU-box round evidence: GPU suite; config-3 bench (headline line, CPU
# baseline, stage pass); rocprofv3 kernel trace + stats of the same bench;
# HBM traffic PMC passes (one counter per pass); config-4 and config-5
# benches.  Every GPU step under its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; echo "rocprof exit $rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err
  rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || exit $rc
done
cd $R
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; [ $rc -eq 0 ] || { echo "bench c4 failed $rc"; tail -30 gpurun_out/bench_c4.err; exit $rc; }
cat gpurun_out/bench_c4.json
timeout -k 10 400 python bench.py --config 5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
rc=$?; [ $rc -eq 0 ] || { echo "bench c5 failed $rc"; tail -30 gpurun_out/bench_c5.err; exit $rc; }
cat gpurun_out/bench_c5.json
