#!/bin/bash
# round 4 (w): config 4's k_act_seq, per batch: complex steps, chain
# windows, wave fallbacks and phase clocks (debug queues, DMC_DEBUG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/round_debug.py --config4 > gpurun_out/r04w_actseq.txt 2>&1 || { tail -20 gpurun_out/r04w_actseq.txt; exit 1; }
grep -E "act_seq" gpurun_out/r04w_actseq.txt | tail -30
