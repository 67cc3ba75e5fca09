#!/bin/bash
# round 4 (v): k_remit's per-block phase clocks and per-candidate staging /
# walk durations on config 3's workload (DMC_EMIT_CLOCKS, debug rounds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
DMC_LIB=${DMC_LIB:-} DMC_EMIT_CLOCKS=1 timeout -k 10 300 python tools/round_debug.py --bench > gpurun_out/r04v_emit_clocks.txt 2>&1 || { tail -20 gpurun_out/r04v_emit_clocks.txt; exit 1; }
grep -E "emit clock|emit cand|===" gpurun_out/r04v_emit_clocks.txt | tail -36
