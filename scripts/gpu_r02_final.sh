#!/bin/bash
# round-2 final evidence at HEAD: the whole -m gpu suite, smoke(), the default
# bench command (CPU baseline included), rocprofv3 kernel stats of the same
# command (timed steps extracted), separate FETCH_SIZE / WRITE_SIZE passes
# (calibrated traffic per stage), config-4 and config-5 bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/fin_pytest.log; tail -2 gpurun_out/fin_pytest.log
[ $rc -eq 0 ] || { grep -n "FAIL\|Error" gpurun_out/fin_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/fin_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err
rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/fin_bench.err; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/fin_bench.json')); print('bench', d['ms_per_step'], d['value']/1e6, d['roofline']['frac'], d['cpu_baseline']['value'])"
# kernel stats of the default bench command (stage pass off: the last 20 steps are the timed ones)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fin_stats -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-profile > gpurun_out/fin_stats_bench.json 2> gpurun_out/fin_stats_bench.err
rc=$?; echo "stats exit $rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/fin_stats_bench.err; exit $rc; }
python tools/stepstats.py gpurun_out/fin_stats/run_kernel_trace.csv 20 > gpurun_out/fin_kernel_stats_timed.csv
# PMC traffic (one counter group per pass)
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err
  rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_$C.err; exit $rc; }
done
python tools/pmc_traffic.py --out gpurun_out/fin_traffic.json
timeout -k 10 500 python bench.py --config 4 > gpurun_out/fin_bench_c4.json 2> gpurun_out/fin_bench_c4.err
rc=$?; echo "config4 exit $rc"; [ $rc -eq 0 ] || { tail -10 gpurun_out/fin_bench_c4.err; exit $rc; }
timeout -k 10 500 python bench.py --config 5 > gpurun_out/fin_bench_c5.json 2> gpurun_out/fin_bench_c5.err
rc=$?; echo "config5 exit $rc"; [ $rc -eq 0 ] || { tail -10 gpurun_out/fin_bench_c5.err; exit $rc; }
python -c "
import json
for f in ('fin_bench_c4', 'fin_bench_c5'):
    d = json.load(open('gpurun_out/%s.json' % f)); print(f, d['ms_per_step'], d['value']/1e6, d['roofline'] and d['roofline']['kernel'], d['roofline'] and d['roofline']['frac'], d['cpu_baseline'] and d['cpu_baseline']['value'])"
