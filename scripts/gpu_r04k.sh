#!/bin/bash
# round 4 (k): the pick's histogram load ahead of the key loads (base)
# against the previous order (oldpick), and 64-thread rank blocks (r64):
# exact-trace parity of base and r64 via DMC_LIB, then the A/B timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${PARITY_VARIANTS:-base r64}; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 500 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or tied_rank or bench_shaped" > gpurun_out/r04k_par_$v.log 2>&1 || { echo "par_$v failed"; tail -30 gpurun_out/r04k_par_$v.log; exit 1; }
  echo "par_$v ok: $(tail -1 gpurun_out/r04k_par_$v.log)"
done &&
VARIANTS="${VARIANTS:-base oldpick r64}" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_variants.sh > gpurun_out/r04k_variants.log 2>&1; rc=$?; cat gpurun_out/r04k_variants.log; exit $rc
