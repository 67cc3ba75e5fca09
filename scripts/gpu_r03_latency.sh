#!/bin/bash
# round 3 single-call latency (tests/cpp/latency.cc, 2,000 add + pull rounds):
# the serve path (facade and engine legs) at 10K / 100K / 1M clients with
# the oracle beside it, and the single-op kernels at 1M for comparison
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
L=tests/cpp/latency
timeout -k 10 120 $L 10000 2000 --serve > gpurun_out/r03_latency_10k_serve.json &&
timeout -k 10 180 $L 100000 2000 --serve > gpurun_out/r03_latency_100k_serve.json &&
timeout -k 10 400 $L 1048576 2000 --serve > gpurun_out/r03_latency_1m_serve.json &&
timeout -k 10 200 $L 1048576 2000 --no-facade --no-oracle > gpurun_out/r03_latency_1m_kernels.json &&
cat gpurun_out/r03_latency_*.json
