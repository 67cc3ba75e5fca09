#!/bin/bash
# captured activation adds: config-4 parity, then config-4 A/B (HEAD vs working tree)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "config4 or churn or activation or device or undercut or chunks" > gpurun_out/c4ab_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/c4ab_pytest.log; [ $rc -eq 0 ] || { grep -n "Error\|assert\|FAIL" gpurun_out/c4ab_pytest.log | head; exit $rc; }
cp dmclock_amd/libdmclock_gpu.so /tmp/keep.so
for round in 1 2; do
for v in head cur; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > gpurun_out/c4ab_$v.json 2> gpurun_out/c4ab_$v.err || { tail -5 gpurun_out/c4ab_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c4ab_$v.json')); print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()})"
done
done
cp /tmp/keep.so dmclock_amd/libdmclock_gpu.so
