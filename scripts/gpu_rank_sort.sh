#!/bin/bash
# sorted rank bins (k_rrank's bitonic path for bins of > 192 records): the
# rank parity tests (tied bins, config 4 at 64K and 1M clients), then A/B of
# config 4 and config 3 against HEAD (variants head / cur)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_device_parity.py tests/test_gpu_parity.py -k "${TESTS_K:-config4 or tied or bench_shaped or activation}" > gpurun_out/rs_tests.log 2>&1
rc=$?; tail -3 gpurun_out/rs_tests.log; [ $rc = 0 ] || exit $rc
VARIANTS="head cur" ROUNDS=2 BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh &&
VARIANTS="head cur" ROUNDS=1 bash scripts/gpu_variants.sh
