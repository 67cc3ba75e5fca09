#!/bin/bash
# Round 2, first GPU call: the GPU suite (new device-API parity at config 3
# full size and config 4 at 64K, world-2 device trackers, tied bins with
# engine counters), the tie study, the config-3 bench (new bytes model and
# engine counters), a 2-rank rehearsal of bench.py --gpus 2 on one GPU
# (gloo), and config 4.  Every GPU step has its own limit; the first failure
# ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/tie_study.py --out gpurun_out/tie_study.json > gpurun_out/tie_study.log 2>&1
rc=$?; tail -4 gpurun_out/tie_study.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; [ $rc -eq 0 ] || { echo "bench failed $rc"; tail -30 gpurun_out/bench.err; exit $rc; }
cat gpurun_out/bench.json
BENCH_SHARE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --clients 262144 --batch 16384 --steps 10 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/bench_w2.json 2> gpurun_out/bench_w2.err
rc=$?; [ $rc -eq 0 ] || { echo "bench w2 failed $rc"; tail -30 gpurun_out/bench_w2.err; exit $rc; }
cat gpurun_out/bench_w2.json
timeout -k 10 400 python bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; [ $rc -eq 0 ] || { echo "bench c4 failed $rc"; tail -30 gpurun_out/bench_c4.err; exit $rc; }
cat gpurun_out/bench_c4.json
