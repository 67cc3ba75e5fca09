#!/bin/bash
# config 3 at several batch sizes (adds = pulls per step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for B in 16384 32768 65536 131072 262144; do
  timeout -k 10 300 python bench.py --batch $B --no-cpu-baseline --steps 20 > gpurun_out/sweep_$B.json 2> gpurun_out/sweep_$B.err || { tail -5 gpurun_out/sweep_$B.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], round(d['value']/1e6,1), 'Mops/s', d['stages_ms_per_step'], d['engine_counters']['radix_rounds'], d['engine_counters']['max_bin'])" gpurun_out/sweep_$B.json $B
done
