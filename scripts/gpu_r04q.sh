#!/bin/bash
# round 4 (q): delayed tags through k_chain_scan -- the chain's scan from
# registers (dreg) against a reload of the slot's ScanRec (dreload)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in dcur dfront dprint; do
DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "pipelined_calls and delayed" > gpurun_out/r04q_$v.log 2>&1; echo "$v rc $?: $(tail -1 gpurun_out/r04q_$v.log)"
done
