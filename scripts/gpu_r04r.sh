#!/bin/bash
# round 4 (r): built with -fno-strict-aliasing (no fence): the pipelined,
# exact-trace, fused and Reject parity tests, then A/B against the strict
# aliasing build with the fence (old)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 800 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "pipelined or exact_trace or fused or reject or bench_shaped" > gpurun_out/r04r_par.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/r04r_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04r_par.log)"
VARIANTS="${VARIANTS:-base old}" ROUNDS=3 BENCH_ARGS="--no-profile --steps 40" timeout -k 10 600 bash scripts/gpu_variants.sh > gpurun_out/r04r_variants.log 2>&1; rc=$?; cat gpurun_out/r04r_variants.log; exit $rc
