#!/bin/bash
# round 4 (i): where the step's time beyond its kernels goes -- host time
# per call (BENCH_HOST_TIMING) with and without pipelining, graphs, and a
# runtime trace of the pipelined bench (API call durations)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in pipe nopipe nographs; do
  flag=""; [ $v = nopipe ] && flag="--no-pipeline"; [ $v = nographs ] && flag="--no-graphs"
  BENCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --steps 40 $flag > gpurun_out/r04i_b_$v.json 2> gpurun_out/r04i_b_$v.err || { echo "bench $v failed"; tail -20 gpurun_out/r04i_b_$v.err; exit 1; }
  echo "$v: $(grep 'host time' gpurun_out/r04i_b_$v.err)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d $R/gpurun_out/r04i_rt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps 10 > gpurun_out/r04i_rt.log 2>&1 || { echo "rt trace failed"; tail -5 gpurun_out/r04i_rt.log; exit 1; }
ls gpurun_out/r04i_rt
VARIANTS="${VARIANTS:-base rpnarrow}" ROUNDS=3 timeout -k 10 600 bash scripts/gpu_variants.sh > gpurun_out/r04i_variants.log 2>&1; rc=$?; cat gpurun_out/r04i_variants.log; exit $rc
