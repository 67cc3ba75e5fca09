#!/bin/bash
# round 4 (ad): queue groups' thresholds and rank-bin tables picked by one
# block per table (k_rpick_m, pm1) vs by every k_remit_m block (pm0): group
# parity through pm1, then config 5 alternated, with kernel stats of pm1
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
DMC_LIB=$R/dmclock_amd/variants/pm1.so timeout -k 10 900 $T tests/test_group.py tests/test_concurrency.py > gpurun_out/r04ad_pytest.log 2>&1 || { tail -20 gpurun_out/r04ad_pytest.log; exit 1; }
tail -1 gpurun_out/r04ad_pytest.log
for round in 1 2; do
for v in pm0 pm1; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-profile > gpurun_out/r04ad_c5_$v.json 2> gpurun_out/r04ad_c5_$v.err || { tail -5 gpurun_out/r04ad_c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04ad_c5_$v.json').read().strip().splitlines()[-1]); print('c5 $v', d['ms_per_step'], d['value'])"
done
done
DMC_LIB=$R/dmclock_amd/variants/pm1.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r04ad_prof -o run --output-format csv -- python3 $R/bench.py --config 5 --no-cpu-baseline --no-profile --steps 6 --warmup 2 > gpurun_out/r04ad_prof.log 2>&1 || { tail -5 gpurun_out/r04ad_prof.log; exit 1; }
python tools/stepstats.py gpurun_out/r04ad_prof/run_kernel_trace.csv 6 > gpurun_out/r04ad_c5_kernel_stats_timed.csv
