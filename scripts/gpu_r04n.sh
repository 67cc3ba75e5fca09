#!/bin/bash
# round 4 (n): k_chain_scan's scan side, 2 / 4 / 8 slots per thread
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
VARIANTS="${VARIANTS:-base cs2 cs8}" ROUNDS=3 BENCH_ARGS="--no-profile --steps 40" timeout -k 10 600 bash scripts/gpu_variants.sh > gpurun_out/r04n_variants.log 2>&1; rc=$?; cat gpurun_out/r04n_variants.log; exit $rc
