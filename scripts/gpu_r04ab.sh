#!/bin/bash
# round 4 (ab): thresholds and rank-bin tables picked once per round by
# k_rhist's last block: queue groups (pm1, the default) vs every k_remit
# block picking (pm0); single-table rounds pre-picked (pp1) vs not (pm1):
# group and single-table parity through each build, then config 5 and
# config 3 alternated on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
DMC_LIB=$R/dmclock_amd/variants/pm1.so timeout -k 10 900 $T tests/test_group.py tests/test_concurrency.py > gpurun_out/r04ab_pytest_pm1.log 2>&1 || { tail -20 gpurun_out/r04ab_pytest_pm1.log; exit 1; }
tail -1 gpurun_out/r04ab_pytest_pm1.log
DMC_LIB=$R/dmclock_amd/variants/pp1.so timeout -k 10 900 $T tests/test_device_parity.py tests/test_gpu_parity.py > gpurun_out/r04ab_pytest_pp1.log 2>&1 || { tail -20 gpurun_out/r04ab_pytest_pp1.log; exit 1; }
tail -1 gpurun_out/r04ab_pytest_pp1.log
for round in 1 2; do
for v in pm0 pm1; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-profile > gpurun_out/r04ab_c5_$v.json 2> gpurun_out/r04ab_c5_$v.err || { tail -5 gpurun_out/r04ab_c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04ab_c5_$v.json').read().strip().splitlines()[-1]); print('c5 $v', d['ms_per_step'], d['value'])"
done
done
VARIANTS="pm1 pp1" ROUNDS=2 timeout -k 10 600 bash scripts/gpu_variants.sh
