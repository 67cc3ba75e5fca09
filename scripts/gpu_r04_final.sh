#!/bin/bash
# round 4 final evidence at HEAD: the -m gpu suite, smoke(), PMC traffic
# passes, the default bench line, kernel stats of the same bench command
# (timed steps), config 4, config 5 (queue group), single-call latency;
# outputs gpurun_out/r04f_* (copied into profiles/ afterwards).
# PART=a: suite + smoke + PMC + bench + stats; PART=b: configs 4/5 + latency;
# PART=c: config 5 and its kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r04f_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r04f_$n.log | cut -c1-300
  return $rc
}
if [ "${PART:-a}" = a ]; then
run suite 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread &&
run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" &&
bash scripts/gpu_pmc.sh &&
python tools/pmc_traffic.py --out gpurun_out/traffic_r04f.json > gpurun_out/r04f_traffic.log 2>&1 &&
run bench 300 python bench.py --traffic gpurun_out/traffic_r04f.json &&
run stats 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04f_prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile &&
python tools/stepstats.py gpurun_out/r04f_prof/run_kernel_trace.csv 20 > gpurun_out/r04f_kernel_stats_timed.csv
elif [ "${PART}" = c ]; then
run c5 400 python bench.py --config 5 --no-cpu-baseline &&
run c5stats 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04f_c5prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-profile --steps 6 --warmup 2 &&
python tools/stepstats.py gpurun_out/r04f_c5prof/run_kernel_trace.csv 6 > gpurun_out/r04f_c5_kernel_stats_timed.csv
else
run c4 400 python bench.py --config 4 &&
run c4stats 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04f_c4prof -o run --output-format csv -- python3 $R/bench.py --config 4 --no-cpu-baseline --no-profile &&
python tools/stepstats.py gpurun_out/r04f_c4prof/run_kernel_trace.csv 20 > gpurun_out/r04f_c4_kernel_stats_timed.csv &&
run c5 400 python bench.py --config 5 --no-cpu-baseline &&
run c5stats 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04f_c5prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-profile --steps 6 --warmup 2 &&
run lat1m 300 tests/cpp/latency 1048576 2000 --serve &&
run lat6q 300 tests/cpp/latency 100000 3000 --serve --no-oracle --no-facade --queues 6
fi
