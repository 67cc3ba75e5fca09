#!/bin/bash
# emit phase clocks (debug) at the current engine
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
DMC_DEBUG=1 DMC_EMIT_CLOCKS=1 timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/eclk.json 2> gpurun_out/eclk.err || { tail -5 gpurun_out/eclk.err; exit 1; }
grep "emit clock\|emit cand" gpurun_out/eclk.err | tail -7
