#!/bin/bash
# round 4 (m): host cost of the eager pipelined step (runtime API trace of
# the timed steps) and the bench's host timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
BENCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 40 > gpurun_out/r04m_b.json 2> gpurun_out/r04m_b.err || { tail -5 gpurun_out/r04m_b.err; exit 1; }
grep 'host time' gpurun_out/r04m_b.err; python -c "import json; d=json.loads(open('gpurun_out/r04m_b.json').read().strip().splitlines()[-1]); print(d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace -d $R/gpurun_out/r04m_rt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 20 > gpurun_out/r04m_rt.log 2>&1 || { tail -5 gpurun_out/r04m_rt.log; exit 1; }
echo done
