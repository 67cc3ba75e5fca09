#!/bin/bash
# round 4 (h): pipelined dmc_add_pull_batch_device calls (DMC_OPT_PIPELINE):
# their parity tests (incl. the gate's redo path), then bench.py with and
# without pipelining, alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 600 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "pipelined or fused or exact_trace or reject" > gpurun_out/r04h_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/r04h_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04h_par.log)"
for v in pipe nopipe pipe nopipe; do
  flag=""; [ $v = nopipe ] && flag="--no-pipeline"
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 40 $flag > gpurun_out/r04h_b_$v.json 2> gpurun_out/r04h_b_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/r04h_b_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04h_b_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], d['engine_counters']['decisions'])"
done
