#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, each under
# a hard limit), plus the list of available counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1; echo "list exit $?"
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$tag -o run --output-format csv -- python3 $R/bench.py --steps 6 --warmup 2 --prof-steps 0 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/pmc_$tag.json 2> $R/gpurun_out/pmc_$tag.err
  rc=$?; echo "pmc $tag exit $rc"; [ $rc -eq 0 ] || { tail -5 $R/gpurun_out/pmc_$tag.err; exit $rc; }
done
