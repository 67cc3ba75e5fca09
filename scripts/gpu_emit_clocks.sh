#!/bin/bash
# k_remit's per-block phase clocks and per-candidate staging / walk times
# (debug build paths of the shipped library, DMC_EMIT_CLOCKS) over bench.py's
# config-3 workload, eager host-API rounds
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
DMC_EMIT_CLOCKS=1 timeout -k 10 300 python tools/round_debug.py --bench > gpurun_out/emit_clocks.log 2>&1
rc=$?
grep -A8 '=== step 5' gpurun_out/emit_clocks.log | grep 'emit' 
exit $rc
