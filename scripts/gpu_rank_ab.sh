#!/bin/bash
# k_rrank's sort threshold (DMC_RANK_SORT_MIN variants s192 / s128 / s64):
# the tied-bin tests on the smallest threshold, then A/B of config 3 and 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
DMC_LIB=$R/dmclock_amd/variants/s64.so timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_device_parity.py -k "tied or bench_shaped or fused_bench or config4" > gpurun_out/rab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/rab_tests.log; [ $rc = 0 ] || exit $rc
VARIANTS="s192 s128 s64" ROUNDS=2 bash scripts/gpu_variants.sh &&
VARIANTS="s192 s128 s64" ROUNDS=1 BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh
