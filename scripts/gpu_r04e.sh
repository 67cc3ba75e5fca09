#!/bin/bash
# round 4 (e): rank / scan launch-shape variants (parity via DMC_LIB, then
# the A/B timing that rejects a wrong-result build), and the single-call
# latency of the serve path (answer before re-summary) incl. six serving
# queues driven round-robin from one thread
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/r04e_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -2 gpurun_out/r04e_$n.log | cut -c1-400
  return $rc
}
run clocks 300 bash scripts/gpu_emit_clocks.sh &&
cp gpurun_out/emit_clocks.log gpurun_out/r04e_emit_clocks_full.log &&
for v in base e512s base e512s; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-profile --steps 10 > gpurun_out/r04e_c5_$v.json 2> gpurun_out/r04e_c5_$v.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04e_c5_$v.json')); print('c5 $v', d['ms_per_step'], d['decisions_per_s'])"
done &&
run lat1m 300 tests/cpp/latency 1048576 2000 --serve &&
run lat6q 300 tests/cpp/latency 100000 3000 --serve --no-oracle --no-facade --queues 6 &&
for v in ${PARITY_VARIANTS:-r128 base}; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so run par_$v 500 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or tied_rank or bench_shaped or churn_activations" || exit 1
done &&
VARIANTS="${VARIANTS:-base nodpp r128 sc2 st2}" ROUNDS=2 timeout -k 10 900 bash scripts/gpu_variants.sh > gpurun_out/r04e_variants.log 2>&1; rc=$?; cat gpurun_out/r04e_variants.log; exit $rc
