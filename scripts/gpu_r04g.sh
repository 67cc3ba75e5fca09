#!/bin/bash
# round 4 (g): wave scans / sums on the DPP network (k_remit compaction,
# pick, rank, hist) against the shuffle loops: parity of both builds via
# DMC_LIB, then the A/B timing (decision counts checked against base); first
# the activation tests (AtLimit::Reject resolved on the device, k_act_hard)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so"; exit 3; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_device_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "reject or activation or churn or config4" > gpurun_out/r04g_act.log 2>&1 || { echo "act tests failed"; tail -40 gpurun_out/r04g_act.log; exit 1; }
echo "act ok: $(tail -1 gpurun_out/r04g_act.log)"; grep "predicted" gpurun_out/r04g_act.log | head
for v in ${PARITY_VARIANTS:-base wshfl}; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 500 python -u -m pytest tests/test_device_parity.py tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "exact_trace or tied_rank or bench_shaped or churn_activations" > gpurun_out/r04g_par_$v.log 2>&1 || { echo "par_$v failed"; tail -30 gpurun_out/r04g_par_$v.log; exit 1; }
  echo "par_$v ok: $(tail -1 gpurun_out/r04g_par_$v.log)"
done &&
VARIANTS="${VARIANTS:-base wshfl scandpp}" ROUNDS=3 timeout -k 10 900 bash scripts/gpu_variants.sh > gpurun_out/r04g_variants.log 2>&1; rc=$?; cat gpurun_out/r04g_variants.log; exit $rc
