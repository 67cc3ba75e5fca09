#!/bin/bash
# GPU-box: multi-server parity test, then config-5 bench lines (small, full).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || { echo "stale .so: build first"; exit 3; }
timeout -k 10 300 python -u -m pytest tests/test_multiserver.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ms.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ms.log; tail -5 gpurun_out/pytest_ms.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 5 --clients 262144 --steps 16 --warmup 4 --epoch-steps 8 > gpurun_out/bench5_small.json 2> gpurun_out/bench5_small.err
rc=$?; [ $rc -eq 0 ] || { echo "bench5 small failed $rc"; tail -30 gpurun_out/bench5_small.err; exit $rc; }
cat gpurun_out/bench5_small.json
timeout -k 10 400 python bench.py --config 5 ${BENCH_ARGS} > gpurun_out/bench5.json 2> gpurun_out/bench5.err
rc=$?; [ $rc -eq 0 ] || { echo "bench5 failed $rc"; tail -30 gpurun_out/bench5.err; exit $rc; }
cat gpurun_out/bench5.json
