#!/bin/bash
# round 3 final evidence at HEAD: the -m gpu suite, smoke(), PMC traffic
# passes, the default bench line, kernel stats of the same bench command
# (timed steps), config 4, config 5 (4 and 8 hardware queues); outputs
# gpurun_out/r03f_* (copied into profiles/ afterwards)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r03f_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r03f_$n.log | cut -c1-300
  return $rc
}
run suite 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread &&
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
bash scripts/gpu_pmc.sh &&
python tools/pmc_traffic.py --out gpurun_out/traffic_r03f.json > gpurun_out/r03f_traffic.log 2>&1 &&
run bench 300 python bench.py --traffic gpurun_out/traffic_r03f.json &&
run stats 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03f_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile &&
python tools/stepstats.py gpurun_out/r03f_prof/run_kernel_trace.csv 20 > gpurun_out/r03f_kernel_stats_timed.csv &&
run c4 400 python bench.py --config 4 &&
run c5 500 python bench.py --config 5 --no-cpu-baseline &&
GPU_MAX_HW_QUEUES=8 run c5hq8 500 python bench.py --config 5 --no-cpu-baseline
