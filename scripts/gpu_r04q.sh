#!/bin/bash
# round 4 (q): eager_delayed pipelined parity with the add chain then the
# scan (noover) -- is the failure the merged launch's?
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
DMC_LIB=$R/dmclock_amd/variants/noover.so timeout -k 10 300 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "pipelined_calls and delayed" > gpurun_out/r04q_noover.log 2>&1; echo "noover rc $?: $(tail -1 gpurun_out/r04q_noover.log)"
