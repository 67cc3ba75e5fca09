#!/bin/bash
# two-rank rehearsals on the one-GPU box at the round's final code (both
# ranks on GPU 0, gloo): config 3 at 256K clients per rank, and config 5
# with 2 servers per rank (the epoch all-reduce staged through host memory)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export BENCH_SHARE_DEVICE=1
timeout -k 10 400 python bench.py --gpus 2 --clients 262144 --batch 16384 --no-cpu-baseline > gpurun_out/r03_bench_2rank_rehearsal.log 2>&1 &&
grep '^{"metric"' gpurun_out/r03_bench_2rank_rehearsal.log | tail -1 | cut -c1-300 &&
timeout -k 10 500 python bench.py --config 5 --gpus 2 --servers 2 --no-cpu-baseline > gpurun_out/r03_config5_2rank_rehearsal.log 2>&1 &&
grep '^{"metric"' gpurun_out/r03_config5_2rank_rehearsal.log | tail -1 | cut -c1-300
