#!/bin/bash
# GPU-box: HBM traffic counters for the bench's kernels, one counter per pass
# (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: never in one pass), each pass
# under its own hard time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so: build first"; exit 3; }
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err
  rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || exit $rc
done
