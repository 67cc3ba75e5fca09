#!/bin/bash
# round 4 (b): the -m gpu tests touched since r04a (lagged exchange), a
# kernel trace of the config-5 queue-group bench, then the emit block-size
# variants (test_bench_exact_trace_parity via DMC_LIB + the A/B timing)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r04b_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r04b_$n.log | cut -c1-300
  return $rc
}
run ms 400 python -u -m pytest tests/test_multiserver.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread &&
run c5prof 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04b_c5prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-profile --steps 6 --warmup 2 &&
for v in e512 e512s e256; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so run exact_$v 400 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or unset_phase" || exit 1
done &&
VARIANTS="${VARIANTS:-base e512 e512s e256}" ROUNDS=2 timeout -k 10 900 bash scripts/gpu_variants.sh > gpurun_out/r04b_variants.log 2>&1; rc=$?; cat gpurun_out/r04b_variants.log; exit $rc
