#!/bin/bash
# k_act_seq's window / wave-step parameters (DMC_ACT_WAVE_BELOW / _LEN
# variants): activation parity on two variants, then A/B of config 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for v in a64_256 a2_64; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_device_parity.py tests/test_gpu_parity.py -k "config4 or activation or churn" > gpurun_out/act_$v.log 2>&1
  rc=$?; echo "$v"; tail -1 gpurun_out/act_$v.log; [ $rc = 0 ] || exit $rc
done
VARIANTS="a8_64 a8_256 a64_256 a2_64" ROUNDS=2 BENCH_ARGS="--config 4" bash scripts/gpu_variants.sh
