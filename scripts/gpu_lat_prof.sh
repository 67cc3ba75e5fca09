#!/bin/bash
# kernel times of the single-op path (latency tool, engine leg)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 10000 1048576; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/latprof_$n -o lat -- tests/cpp/latency $n 2000 --no-facade --no-oracle > gpurun_out/latprof_$n.log 2>&1 || { tail -20 gpurun_out/latprof_$n.log; exit 1; }
  tail -1 gpurun_out/latprof_$n.log
done
