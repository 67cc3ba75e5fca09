#!/bin/bash
# config 5: default hardware queues (4) vs 8 (one per server queue's stream)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for round in 1 2; do
for hq in 4 8; do
  GPU_MAX_HW_QUEUES=$hq timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5hq_$hq.json 2> gpurun_out/c5hq_$hq.err || { tail -5 gpurun_out/c5hq_$hq.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/c5hq_$hq.json')); print('hwq $hq', d['ms_per_step'], round(d['value']/1e6))"
done
done
