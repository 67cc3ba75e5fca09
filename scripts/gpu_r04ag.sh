#!/bin/bash
# round 4 (ag): the final build's serve path once more on a fresh box: the
# serve, facade and multi-server tests twice, and C-ABI latency at 10K and
# 100K clients (smaller groups than 1M's)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_single_op.py tests/test_facade_cpp.py tests/test_multiserver.py tests/test_gpu_parity.py -k "serve or facade or kat or multiserver" > gpurun_out/r04ag_pytest_$i.log 2>&1 || { tail -20 gpurun_out/r04ag_pytest_$i.log; exit 1; }
tail -1 gpurun_out/r04ag_pytest_$i.log
done
for n in 10000 100000; do
timeout -k 10 300 tests/cpp/latency $n 2000 --serve > gpurun_out/r04ag_lat_$n.txt 2>&1 || { tail -5 gpurun_out/r04ag_lat_$n.txt; exit 1; }
tail -1 gpurun_out/r04ag_lat_$n.txt
done
