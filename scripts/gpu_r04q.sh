#!/bin/bash
# round 4 (q): delayed tags through k_chain_scan with the chain's writes
# fenced before the slot's walk
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "pipelined_calls" > gpurun_out/r04q_fence.log 2>&1; echo "fence rc $?: $(tail -1 gpurun_out/r04q_fence.log)"
