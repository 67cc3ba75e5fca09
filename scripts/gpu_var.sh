#!/bin/bash
# run-to-run variance of the default bench line (and a longer run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/var_$i.json 2> gpurun_out/var_$i.err || { tail -5 gpurun_out/var_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_$i.json')); print('run $i ms_per_step', d['ms_per_step'])"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 200 > gpurun_out/var_long.json 2> gpurun_out/var_long.err || { tail -5 gpurun_out/var_long.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/var_long.json')); print('200 steps ms_per_step', d['ms_per_step'])"
