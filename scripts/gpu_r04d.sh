#!/bin/bash
# round 4 (d): heap-order tests, the group tests (fused tracker fill), the
# config-5 bench and its kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r04d_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r04d_$n.log | cut -c1-300
  return $rc
}
run heap 700 python -u -m pytest tests/test_group.py tests/test_concurrency.py -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread &&
run c5 300 python bench.py --config 5 --no-cpu-baseline &&
run c5prof 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04d_c5prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-profile --steps 6 --warmup 2
