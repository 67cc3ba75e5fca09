#!/bin/bash
# round 4 (ai): the activation inputs gathered by k_act_keys (no k_act_inputs launch; anew) vs
# HEAD (abase): activation parity tests, the per-batch probe, then config 4
# alternated on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_device_parity.py tests/test_gpu_parity.py tests/test_device_api.py -k "activ or config4 or churn or reject" > gpurun_out/r04ai_pytest.log 2>&1 || { tail -20 gpurun_out/r04ai_pytest.log; exit 1; }
tail -2 gpurun_out/r04ai_pytest.log
timeout -k 10 300 python tools/round_debug.py --config4 > gpurun_out/r04ai_actseq.txt 2>&1 || { tail -20 gpurun_out/r04ai_actseq.txt; exit 1; }
grep -E "act_seq" gpurun_out/r04ai_actseq.txt | tail -6
for round in 1 2; do
for v in abase anew; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/r04ai_c4_$v.json 2> gpurun_out/r04ai_c4_$v.err || { tail -5 gpurun_out/r04ai_c4_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04ai_c4_$v.json').read().strip().splitlines()[-1]); print('c4 $v', d['ms_per_step'], d['engine_counters']['decisions'], {k: round(x*1e3,1) for k, x in d['stages_ms_per_step'].items()})"
done
done
