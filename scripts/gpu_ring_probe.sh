#!/bin/bash
# TLB-reach probe: the default bench with ring capacities 64 / 32 / 16
# (the ring region is N x Q x 64 B: 4 / 2 / 1 GiB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for round in 1 2; do
for q in 64 32 16; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --ring $q > gpurun_out/ring_$q.json 2> gpurun_out/ring_$q.err || { tail -5 gpurun_out/ring_$q.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ring_$q.json')); print('ring $q', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()})"
done
done
