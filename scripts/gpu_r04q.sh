#!/bin/bash
# round 4 (q): is the delayed-mode failure strict aliasing (the cursor
# word stored through a uint64_t pointer, its fields loaded as ScanRec
# members)?  no fence, with and without -fno-strict-aliasing
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in nofence nofence_nsa; do
DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "pipelined_calls and delayed" > gpurun_out/r04q_$v.log 2>&1; echo "$v rc $?: $(tail -1 gpurun_out/r04q_$v.log)"
done
