#!/bin/bash
# A/B on one box: graph instances alternated (default) / not, early summary off
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
b() {
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -5 gpurun_out/ab_$1.err; exit 1; }
  python -c "import json; a=json.load(open('gpurun_out/ab_$1.json')); print('$1', a['ms_per_step'], a['engine_counters']['graph_replays'])"
}
for i in 1 2; do
  b flip_$i
  DMC_NO_GRAPH_FLIP=1 b noflip_$i
  DMC_NO_GRAPH_FLIP=1 DMC_NO_EARLY_SUMMARY=1 b none_$i
done
