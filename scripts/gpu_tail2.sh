#!/bin/bash
# Tail timings: the atomic-read build and a plain-read build (measurement).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for v in tail tailp; do
  cp dmclock_amd/variants/$v.so dmclock_amd/libdmclock_gpu.so
  DMC_DEBUG=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/$v.json 2> gpurun_out/$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v bench failed $rc"; tail -30 gpurun_out/$v.err; exit $rc; }
  echo "== $v"; grep "dmc tails" gpurun_out/$v.err | tail -4
done
