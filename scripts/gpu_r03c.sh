#!/bin/bash
# round 3: the -m gpu suite, the default bench line, kernel stats of the
# same bench command (timed steps), config 5 with 8 hardware queues
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r03c_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -3 gpurun_out/r03c_$n.log
  return $rc
}
run suite 1000 $PT tests -m gpu &&
run bench 300 python bench.py &&
run stats 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03c_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile &&
python tools/stepstats.py gpurun_out/r03c_prof/run_kernel_trace.csv 20 > gpurun_out/r03c_kernel_stats_timed.csv &&
GPU_MAX_HW_QUEUES=8 run c5hq8 500 python bench.py --config 5 --no-cpu-baseline
