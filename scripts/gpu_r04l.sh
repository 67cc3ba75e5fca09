#!/bin/bash
# round 4 (l): the add chain and the round's scan in one launch, side by
# side (k_chain_scan + k_scan_fix): parity of the paths it runs in (bench
# mode exact trace, pipelined calls, fused calls), then A/B against the
# add kernels followed by k_rscan (noover), and a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 700 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or pipelined or fused or bench_shaped or tied_rank" > gpurun_out/r04l_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/r04l_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04l_par.log)"
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r04l_tr -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 10 > gpurun_out/r04l_tr.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/r04l_tr.log; exit 1; }
VARIANTS="${VARIANTS:-base noover}" ROUNDS=3 BENCH_ARGS="--no-profile" timeout -k 10 600 bash scripts/gpu_variants.sh > gpurun_out/r04l_variants.log 2>&1; rc=$?; cat gpurun_out/r04l_variants.log; exit $rc
