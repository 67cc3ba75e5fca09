#!/bin/bash
# round 4 (t): k_rapply's staged queue positions per candidate (2 / 4 / 8):
# config 4 (activated clients' deep queues walked by the slow path) and
# config 3
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
for v in base as2 as8; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline --no-profile > gpurun_out/r04t_c4_$v.json 2> gpurun_out/r04t_c4_$v.err || { tail -5 gpurun_out/r04t_c4_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04t_c4_$v.json').read().strip().splitlines()[-1]); print('c4 $v', d['ms_per_step'], d['engine_counters']['decisions'])"
done
done
VARIANTS="base as2 as8" ROUNDS=2 BENCH_ARGS="--no-profile --steps 40" timeout -k 10 600 bash scripts/gpu_variants.sh
