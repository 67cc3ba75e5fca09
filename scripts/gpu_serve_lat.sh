#!/bin/bash
# serve-path latency at 1M clients with k_serve's per-call phase stamps
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
DMC_SERVE_TRACE=1 timeout -k 10 300 tests/cpp/latency 1048576 2000 --no-oracle --no-facade --serve > gpurun_out/lat_serve_1m.json 2> gpurun_out/lat_serve.err; rc=$?
cat gpurun_out/lat_serve_1m.json; grep "dmc serve" gpurun_out/lat_serve.err; exit $rc
