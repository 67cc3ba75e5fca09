#!/bin/bash
# config 5 with the fused per-queue call; multiserver tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_multiserver.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/c5b_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 gpurun_out/c5b_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config 5 --no-cpu-baseline > gpurun_out/c5b.json 2> gpurun_out/c5b.err
rc=$?; echo "config5 exit $rc"; [ $rc -eq 0 ] || { tail -10 gpurun_out/c5b.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/c5b.json')); print(d['ms_per_step'], d['value']/1e6, d.get('epoch_delivery_ms'), d['roofline']['frac'])"
