#!/bin/bash
# round 4 (u): serve pull with the reservation top, the ready top and the
# stale-group flag in one block reduction (snew) vs HEAD (sbase): C-ABI pull
# latency, alternated on one box, after the serve parity tests
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_single_op.py tests/test_multiserver.py > gpurun_out/r04u_pytest.log 2>&1 || { tail -20 gpurun_out/r04u_pytest.log; exit 1; }
tail -2 gpurun_out/r04u_pytest.log
for round in 1 2; do
for v in sbase snew; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 300 tests/cpp/latency 1048576 2000 --serve --no-oracle > gpurun_out/r04u_lat_$v.$round.txt 2>&1 || { tail -5 gpurun_out/r04u_lat_$v.$round.txt; exit 1; }
  echo "== $v $round"; grep -i "pull\|p50" gpurun_out/r04u_lat_$v.$round.txt | head -8
done
done
