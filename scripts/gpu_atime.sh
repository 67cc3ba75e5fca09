#!/bin/bash
# Per-candidate apply timings (engine debug mode) over a few bench steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
rm -f /tmp/dmc_bins.bin
DMC_DEBUG=1 DMC_DEBUG_BINS=/tmp/dmc_bins.bin timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/atime.json 2> gpurun_out/atime.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -20 gpurun_out/atime.err; exit $rc; }
python tools/apply_timing.py /tmp/dmc_bins.bin | tail -8
