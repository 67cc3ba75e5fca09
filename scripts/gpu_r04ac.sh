#!/bin/bash
# round 4 (ac): with the groups' tables pre-picked, k_remit at 512 threads
# (79.6 KB LDS: two blocks per CU; e512) vs 1024 (base): group and
# exact-trace parity through e512, then config 5 and config 3 alternated
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
DMC_LIB=$R/dmclock_amd/variants/e512.so timeout -k 10 900 $T tests/test_group.py tests/test_concurrency.py tests/test_device_parity.py -k "group or concurrent or exact_trace" > gpurun_out/r04ac_pytest.log 2>&1 || { tail -20 gpurun_out/r04ac_pytest.log; exit 1; }
tail -1 gpurun_out/r04ac_pytest.log
for round in 1 2; do
for v in base e512; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-profile > gpurun_out/r04ac_c5_$v.json 2> gpurun_out/r04ac_c5_$v.err || { tail -5 gpurun_out/r04ac_c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04ac_c5_$v.json').read().strip().splitlines()[-1]); print('c5 $v', d['ms_per_step'], d['value'])"
done
done
VARIANTS="base e512" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_variants.sh
