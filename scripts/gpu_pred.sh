#!/bin/bash
# predicted-candidate rounds A/B on the shipped library (DMC_NO_PRED turns
# them off), engine counters and per-stage times shown
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for round in 1 2; do
for v in base pred; do
  if [ $v = base ]; then export DMC_NO_PRED=1; else unset DMC_NO_PRED; fi
  DMC_PRED_LOG=1 timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { tail -5 gpurun_out/var_$v.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); c=d['engine_counters']; print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in d['stages_ms_per_step'].items()}, 'pred', c.get('pred_rounds'), c.get('pred_misses'), 'cand', c['candidates'])"
  grep -c 'pred miss' gpurun_out/var_$v.err
done
done
