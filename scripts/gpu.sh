#!/bin/bash
# The one GPU-box runner: named steps, each under its own time limit, run in
# order; the first failing step ends the call (nothing more touches the GPU).
# Outputs: gpurun_out/$TAG_<step>.{log,json,csv} (copy what is judged into
# profiles/).
#
#   usage: TAG=r05a scripts/gpu.sh STEP [STEP ...]
#   steps:
#     suite            pytest -m gpu, the whole suite ($PYTEST_K narrows it with -k)
#     smoke            __graft_entry__.smoke()
#     bench            bench.py (config 3) with this round's traffic file if present
#     stats            rocprofv3 kernel trace of the bench's timed steps + stepstats
#     pmc              FETCH_SIZE and WRITE_SIZE passes (one counter per pass) and
#                      tools/pmc_traffic.py -> gpurun_out/traffic_$TAG.json
#     c4 / c4stats     bench.py --config 4 / its kernel trace
#     c5 / c5stats     bench.py --config 5 / its kernel trace
#     heap             bench.py --heap-order (tie-exact mode at config 3)
#     lat              tests/cpp/latency at 1M clients (serve path)
#     heaptime         tools/heap_timing.py at $HEAP_N clients (heap order vs oracle)
#     rankbins         tools/rank_bins.py: k_rrank's per-bin clocks over 40 debug rounds
#     probe            tools/rand_probe: random-record read rates (64/128-byte shapes)
#     eclk             k_remit's per-block phase clocks and per-candidate walk times
#                      over a short bench run (DMC_DEBUG rounds, stderr)
#     aclk             k_rapply's slow candidates' clocks over a short bench run
#                      (DMC_DEBUG_BINS dump, tools/apply_clocks.py)
#     variants         $VARIANTS alternated $ROUNDS times (scripts/gpu_variants.sh)
#   $BENCH_ARGS is appended to every bench.py command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-run}
O=gpurun_out/${T}
# (a .so older than its sources ran anyway: the sources were edited after its
# build while this call was queued; the .so is what runs)
python -c "from dmclock_amd import build; import sys; sys.exit(0 if build.up_to_date() else 3)" || echo "warning: the .so is older than its sources"

run() {  # name, seconds, command...
  local n=$1 t=$2; shift 2
  echo "== $n: $*"
  timeout -k 10 $t "$@" > ${O}_$n.log 2>&1
  local rc=$?
  echo "$n exit $rc"; tail -3 ${O}_$n.log | cut -c1-400
  return $rc
}
traffic_arg() {
  [ -f gpurun_out/traffic_$T.json ] && echo "--traffic gpurun_out/traffic_$T.json"
}
prof() {  # name, seconds, steps, bench args...
  local n=$1 t=$2 k=$3; shift 3
  run $n $t rocprofv3 --kernel-trace --stats -d $R/${O}_${n}_prof -o run --output-format csv \
      -- python3 $R/bench.py --no-cpu-baseline --no-profile --steps $k "$@" ${BENCH_ARGS} &&
  python tools/stepstats.py ${O}_${n}_prof/run_kernel_trace.csv $k > ${O}_${n}_kernel_stats_timed.csv &&
  head -12 ${O}_${n}_kernel_stats_timed.csv | cut -c1-160
}

for step in "$@"; do
  case $step in
    suite)
      if [ -n "$PYTEST_K" ]; then
        run suite 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread -k "$PYTEST_K"
      else
        run suite 1100 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 600 --timeout-method thread
      fi || exit 1 ;;
    smoke) run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) run bench 300 python bench.py $(traffic_arg) ${BENCH_ARGS} || exit 1
           grep "^{\"metric\"" ${O}_bench.log | tail -1 > ${O}_bench.json ;;
    stats) prof stats 300 20 || exit 1 ;;
    pmc)
      for C in FETCH_SIZE WRITE_SIZE; do
        ( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err )
        rc=$?; echo "pmc $C exit $rc"; [ $rc -eq 0 ] || exit 1
      done
      python tools/pmc_traffic.py --out gpurun_out/traffic_$T.json > ${O}_traffic.log 2>&1 || { tail -5 ${O}_traffic.log; exit 1; }
      tail -12 ${O}_traffic.log ;;
    c4) run c4 400 python bench.py --config 4 ${BENCH_ARGS} || exit 1
        grep "^{\"metric\"" ${O}_c4.log | tail -1 > ${O}_c4.json ;;
    c4stats) prof c4stats 400 20 --config 4 || exit 1 ;;
    c5) run c5 500 python bench.py --config 5 ${BENCH_ARGS} || exit 1
        grep "^{\"metric\"" ${O}_c5.log | tail -1 > ${O}_c5.json ;;
    c5stats) prof c5stats 400 6 --config 5 --warmup 2 || exit 1 ;;
    heap) run heap 900 python bench.py --heap-order ${BENCH_ARGS} || exit 1
          grep "^{\"metric\"" ${O}_heap.log | tail -1 > ${O}_heap.json ;;
    lat) run lat 300 tests/cpp/latency 1048576 2000 --serve || exit 1 ;;
    heaptime) run heaptime_${HEAP_N:-65536} 600 python -u tools/heap_timing.py ${HEAP_N:-65536} 2 ${HEAP_ARGS} || exit 1 ;;
    variants) bash scripts/gpu_variants.sh || exit 1 ;;
    rankbins) run rankbins 300 python -u tools/rank_bins.py 40 || exit 1 ;;
    probe) run probe 200 tools/rand_probe || exit 1 ;;
    eclk) DMC_DEBUG=1 DMC_EMIT_CLOCKS=1 run eclk 300 python bench.py --steps 3 --warmup 1 \
              --no-cpu-baseline --no-profile ${BENCH_ARGS} || exit 1
          grep -c 'emit clock' ${O}_eclk.log ;;
    aclk) rm -f /tmp/aclk_$T.bin
          DMC_DEBUG=1 DMC_DEBUG_BINS=/tmp/aclk_$T.bin run aclk_bench 300 python bench.py --steps 3 \
              --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} || exit 1
          run aclk 60 python tools/apply_clocks.py /tmp/aclk_$T.bin 4 || exit 1
          cat ${O}_aclk.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
