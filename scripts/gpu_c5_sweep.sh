#!/bin/bash
# GPU-box: config-5 concurrency sweep over servers per GPU, and a kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for S in 1 2 4 8; do
  timeout -k 10 200 python bench.py --config 5 --servers $S --steps 16 --warmup 4 > gpurun_out/c5_s$S.json 2> gpurun_out/c5_s$S.err || { echo "S=$S failed"; tail -20 gpurun_out/c5_s$S.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5_s$S.json'));print($S, d['value']/1e6, d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c5 -o run --output-format csv -- python $R/bench.py --config 5 --servers 8 --steps 8 --warmup 2 > $R/gpurun_out/c5_prof.json 2> $R/gpurun_out/c5_prof.err || { echo "prof failed"; tail -20 $R/gpurun_out/c5_prof.err; exit 1; }
find $R/gpurun_out/prof_c5 -name "*.csv" | head
