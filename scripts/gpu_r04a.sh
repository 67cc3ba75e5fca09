#!/bin/bash
# round 4, first GPU call: the -m gpu suite at HEAD (outcome check, fault
# hook), emit block-size variants A/B (scripts/gpu_variants.sh rejects a
# variant whose decisions differ from the base's), and the 512 / 256-thread
# variants through test_bench_exact_trace_parity via DMC_LIB
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r04a_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r04a_$n.log | cut -c1-300
  return $rc
}
if [ -z "$VARIANTS_ONLY" ]; then
run suite 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread &&
run c5 300 python bench.py --config 5 --no-cpu-baseline &&
run c5sep 300 python bench.py --config 5 --no-cpu-baseline --separate-queues
exit $?
fi
for v in e512 e512s e256; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so run exact_$v 400 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or unset_phase" || exit 1
done &&
VARIANTS="${VARIANTS:-base e512 e512s e256}" ROUNDS=2 timeout -k 10 900 bash scripts/gpu_variants.sh > gpurun_out/r04a_variants.log 2>&1; rc=$?; cat gpurun_out/r04a_variants.log; exit $rc
