#!/bin/bash
# round 4 (p): pipelined-call parity variants (delayed, exact histogram),
# then the configs 4 / 5 and latency evidence (gpu_r04_final.sh PART=b)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "pipelined" > gpurun_out/r04p_par.log 2>&1 || { echo "parity failed"; tail -40 gpurun_out/r04p_par.log; exit 1; }
echo "par ok: $(tail -1 gpurun_out/r04p_par.log)"
PART=b bash scripts/gpu_r04_final.sh
