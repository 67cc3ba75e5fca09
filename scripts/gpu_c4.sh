#!/bin/bash
# config 4 (idle marking + throttled tenants + activations) at 1M clients
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -5 gpurun_out/c4.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/c4.json')); print('c4', d['ms_per_step'], d.get('activations_per_step'), {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()}); print(d.get('engine_counters'))"
