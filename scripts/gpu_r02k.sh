#!/bin/bash
# Round-2 closing checks at HEAD: GPU suite, 2-rank rehearsals (one GPU,
# gloo) of config 3 and config 5, each step under its own limit
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/k_pytest.log; [ $rc -eq 0 ] || exit $rc
BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --clients 262144 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/k_w2.json 2> gpurun_out/k_w2.err
rc=$?; [ $rc -eq 0 ] || { echo "bench w2 failed $rc"; tail -20 gpurun_out/k_w2.err; exit $rc; }
tail -1 gpurun_out/k_w2.json
BENCH_SHARE_DEVICE=1 timeout -k 10 400 python bench.py --config 5 --gpus 2 --servers 2 --steps 32 --warmup 16 --no-cpu-baseline --no-profile > gpurun_out/k_c5w2.json 2> gpurun_out/k_c5w2.err
rc=$?; [ $rc -eq 0 ] || { echo "bench c5 w2 failed $rc"; tail -20 gpurun_out/k_c5w2.err; exit $rc; }
tail -1 gpurun_out/k_c5w2.json
