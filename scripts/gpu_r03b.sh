#!/bin/bash
# round 3: per-round diagnostics (tools/round_debug.py), then the remaining
# GPU tests and a default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread"
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r03b_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -3 gpurun_out/r03b_$n.log
  return $rc
}
run dbg_conc 120 python tools/round_debug.py &&
run dbg_bench 200 python tools/round_debug.py --bench &&
run devpar 600 $PT tests/test_device_parity.py &&
run suite 900 $PT tests -m gpu --deselect tests/test_concurrency.py --deselect tests/test_device_parity.py &&
run bench 300 python bench.py
