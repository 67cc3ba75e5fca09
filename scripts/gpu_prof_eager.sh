#!/bin/bash
# GPU-box: rocprofv3 kernel trace of the bench's stage-timed (eager) pass only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so: build first"; exit 3; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profe -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --prof-steps 5 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/profe_bench.json 2> $R/gpurun_out/profe.err
rc=$?; echo "rocprof exit $rc"; exit $rc
