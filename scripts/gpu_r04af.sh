#!/bin/bash
# round 4 (af): serve kernel with adds served by wave 0 while wave 1 runs the
# previous pull's owed group re-summary (snew) vs HEAD (sbase): the serve and
# facade tests, then C-ABI latency alternated on one box, then one facade run
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
cp dmclock_amd/variants/snew.so dmclock_amd/libdmclock_gpu.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_single_op.py tests/test_facade_cpp.py tests/test_multiserver.py > gpurun_out/r04af_pytest.log 2>&1 || { tail -20 gpurun_out/r04af_pytest.log; exit 1; }
tail -1 gpurun_out/r04af_pytest.log
for round in 1 2; do
for v in sbase snew; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  timeout -k 10 300 tests/cpp/latency 1048576 2000 --serve --no-oracle --no-facade > gpurun_out/r04af_lat_$v.$round.txt 2>&1 || { tail -5 gpurun_out/r04af_lat_$v.$round.txt; exit 1; }
  echo "== $v $round"; tail -1 gpurun_out/r04af_lat_$v.$round.txt | cut -c1-330
done
done
[ -n "$FACADE" ] && { timeout -k 10 300 tests/cpp/latency 1048576 2000 --serve > gpurun_out/r04af_lat_facade_snew.txt 2>&1 && tail -1 gpurun_out/r04af_lat_facade_snew.txt; }; true
