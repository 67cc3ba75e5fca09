#!/bin/bash
# round 4 (aa): the activation chain's wave-stepped stretches: ballots only
# (wbase) vs one activation at a time after two ballots (wseq2), with a
# higher hand-over threshold (wseq2b32) or longer stretches (wseq2l128):
# activation parity of the stepping variant via DMC_LIB, then config 4
# alternated on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
DMC_LIB=$R/dmclock_amd/variants/wseq2l128.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_device_parity.py tests/test_gpu_parity.py tests/test_device_api.py -k "activ or config4 or churn or reject" > gpurun_out/r04aa_pytest.log 2>&1 || { tail -20 gpurun_out/r04aa_pytest.log; exit 1; }
tail -2 gpurun_out/r04aa_pytest.log
for round in 1 2; do
for v in wbase wseq2 wseq2b32 wseq2l128; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/r04aa_c4_$v.json 2> gpurun_out/r04aa_c4_$v.err || { tail -5 gpurun_out/r04aa_c4_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04aa_c4_$v.json').read().strip().splitlines()[-1]); print('c4 $v', d['ms_per_step'], d['engine_counters']['decisions'], {k: round(x*1e3,1) for k, x in d['stages_ms_per_step'].items()})"
done
done
