#!/bin/bash
# round 4 (o): the add chain beside the scan for queue groups
# (k_chain_scan_m): the group / multiserver / concurrency tests, then
# config 5 with and without it
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 900 python -u -m pytest tests/test_group.py tests/test_concurrency.py tests/test_multiserver.py -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread > gpurun_out/r04o_par.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04o_par.log; exit 1; }
echo "tests ok: $(tail -1 gpurun_out/r04o_par.log)"
for v in base noover base noover; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-profile --steps 10 > gpurun_out/r04o_c5_$v.json 2> gpurun_out/r04o_c5_$v.err || { echo "c5 $v failed"; tail -5 gpurun_out/r04o_c5_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04o_c5_$v.json').read().strip().splitlines()[-1]); print('c5 $v', d['ms_per_step'], d['value'])"
done
