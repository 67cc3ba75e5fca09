#!/bin/bash
# round 4 (ae): the final build over 200 timed steps (config 3), and the
# N=2 launch path rehearsed on one card (BENCH_SHARE_DEVICE=1: both ranks on
# device 0, so its rate is not a scaling number)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline --no-profile > gpurun_out/r04ae_200.json 2> gpurun_out/r04ae_200.err || { tail -5 gpurun_out/r04ae_200.err; exit 1; }
tail -1 gpurun_out/r04ae_200.json | cut -c1-400
BENCH_SHARE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/r04ae_n2.json 2> gpurun_out/r04ae_n2.err || { tail -5 gpurun_out/r04ae_n2.err; exit 1; }
tail -1 gpurun_out/r04ae_n2.json | cut -c1-400
