#!/bin/bash
# round-2 evidence: FETCH_SIZE calibration, PMC traffic and kernel stats of
# the config-3 bench, config-5 bench with roofline and CPU baseline
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
# 1. calibration kernels: known bytes, one FETCH_SIZE pass, one trace pass
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/calib_fetch -o run --output-format csv -- $R/tools/fetch_calib > gpurun_out/calib_known.json 2> gpurun_out/calib_fetch.err
rc=$?; echo "calib fetch exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/calib_fetch.err; exit $rc; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/calib_trace -o run --output-format csv -- $R/tools/fetch_calib > /dev/null 2> gpurun_out/calib_trace.err
rc=$?; echo "calib trace exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/calib_trace.err; exit $rc; }
# 2. PMC traffic of the bench (separate passes)
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err
  rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_$C.err; exit $rc; }
done
# 3. kernel stats of the default bench command
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/stats -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > gpurun_out/stats_bench.json 2> gpurun_out/stats_bench.err
rc=$?; echo "stats exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/stats_bench.err; exit $rc; }
# 4. config 5 (one GPU: all server queues on it) with roofline and CPU baseline
timeout -k 10 400 python3 bench.py --config 5 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
rc=$?; echo "config5 exit $rc"; [ $rc -eq 0 ] || { tail -10 gpurun_out/bench_c5.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_c5.json')); print({k: d[k] for k in ('value','unit','ms_per_step','roofline','cpu_baseline') if k in d})"
