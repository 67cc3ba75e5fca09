#!/bin/bash
# per-kernel time of config 4 (rocprofv3 kernel trace, timed steps only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c4prof -o run --output-format csv -- python3 $R/bench.py --config 4 --no-cpu-baseline --no-profile > gpurun_out/c4prof.log 2>&1 || { tail -5 gpurun_out/c4prof.log; exit 1; }
python tools/stepstats.py gpurun_out/c4prof/run_kernel_trace.csv 20 > gpurun_out/c4_kernel_stats.csv && cat gpurun_out/c4_kernel_stats.csv | head -40
