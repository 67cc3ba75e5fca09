#!/bin/bash
# Round-2 perf iteration: the parity tests that cover every engine path
# (KATs, seeded traces in every mode, bench-shaped and full-size device-API
# parity), then the config-3 bench (stage pass), then a rocprofv3 kernel
# trace of an un-staged bench run with per-kernel stats of its timed steps
# and one step's timeline.  Each GPU step under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so: build first"; exit 3; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py tests/test_device_api.py ${TESTS_EXTRA} -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_iter.log; tail -3 gpurun_out/pytest_iter.log
[ $rc -eq 0 ] || { grep -n "Error\|assert" gpurun_out/pytest_iter.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-profile ${BENCH_ARGS} > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err
rc=$?; echo "rocprof exit $rc"; [ $rc -eq 0 ] || exit $rc
cd $R
T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python tools/stepstats.py $T 20 > gpurun_out/kernel_stats_timed.csv && cat gpurun_out/kernel_stats_timed.csv | cut -c1-60,200-
python tools/steps_timeline.py $T 1 > gpurun_out/step_timeline.txt 2>&1; cat gpurun_out/step_timeline.txt
