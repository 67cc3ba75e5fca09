#!/bin/bash
# SQ counters of the bench kernels (one pass, 8 SQ counters)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace -d $R/gpurun_out/pmc_sq -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_sq.json 2> $R/gpurun_out/pmc_sq.err
rc=$?; echo "pmc sq exit $rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_sq.err; exit $rc; }
