#!/bin/bash
# GPU-box: the evidence set for profiles/: GPU tests, the default bench line
# (with the CPU baseline), a rocprofv3 kernel-trace/stats run of the same
# bench (graphs, no stage timers), then the HBM-traffic PMC passes (one
# counter per pass).  Every GPU step has its own limit; the first failure
# ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so: build first"; exit 3; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; echo "rocprof exit $rc"; [ $rc -eq 0 ] || exit $rc
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf $R/gpurun_out/pmc_$C
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err
  rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || exit $rc
done
