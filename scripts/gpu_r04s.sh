#!/bin/bash
# round 4 (s): rank-bin tie flags in O(1) per record (sorted bins): the
# tie / rank tests, config-4 parity, then config 4 and config 3 benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 900 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 400 --timeout-method thread -k "tied or config4 or churn or exact_trace or reject" > gpurun_out/r04s_par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/r04s_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04s_par.log)"
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-profile > gpurun_out/r04s_c4.json 2> gpurun_out/r04s_c4.err || { tail -5 gpurun_out/r04s_c4.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04s_c4.json').read().strip().splitlines()[-1]); print('c4', d['ms_per_step'], d['engine_counters']['max_bin'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 40 > gpurun_out/r04s_c3.json 2> gpurun_out/r04s_c3.err || { tail -5 gpurun_out/r04s_c3.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04s_c3.json').read().strip().splitlines()[-1]); print('c3', d['ms_per_step'])"
