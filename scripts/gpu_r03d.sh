#!/bin/bash
# round 3 evidence at the current code: the default bench line, kernel
# stats of the same bench command (timed steps), PMC traffic passes,
# config 4, config 5 (default and 8 hardware queues)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r03d_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r03d_$n.log | cut -c1-300
  return $rc
}
bash scripts/gpu_pmc.sh &&
python tools/pmc_traffic.py --out gpurun_out/traffic_r03.json > gpurun_out/r03d_traffic.log 2>&1 &&
cp gpurun_out/traffic_r03.json profiles/traffic_r03.json &&
run bench 300 python bench.py &&
run stats 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03d_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile &&
python tools/stepstats.py gpurun_out/r03d_prof/run_kernel_trace.csv 20 > gpurun_out/r03d_kernel_stats_timed.csv &&
run c4 400 python bench.py --config 4 &&
run c5 500 python bench.py --config 5 --no-cpu-baseline &&
GPU_MAX_HW_QUEUES=8 run c5hq8 500 python bench.py --config 5 --no-cpu-baseline
