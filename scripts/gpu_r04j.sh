#!/bin/bash
# round 4 (j): the 8.5 us device-side gap between two replayed graphs --
# pipelined calls with graphs against pipelined calls launched eagerly
# (kernel trace of both: the gaps), parity of the eager pipelined path
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 600 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "pipelined_calls" > gpurun_out/r04j_par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/r04j_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04j_par.log)"
for v in graphs eager graphs eager; do
  flag=""; [ $v = eager ] && flag="--no-graphs"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 40 $flag > gpurun_out/r04j_b_$v.json 2> gpurun_out/r04j_b_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/r04j_b_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04j_b_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['value'], d['engine_counters']['decisions'], d['engine_counters']['fused_calls'])"
  grep 'host time' gpurun_out/r04j_b_$v.err
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r04j_eager -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 10 --no-graphs > gpurun_out/r04j_eager.log 2>&1 || { echo "trace failed"; exit 1; }
echo traced
