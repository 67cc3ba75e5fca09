#!/bin/bash
# GPU-box sweep of the launch-shape variants (scripts/build_variants.sh):
# config-3 bench per variant, the default library restored afterwards.
# Every GPU step under its own limit; the first failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
L=dmclock_amd/libdmclock_gpu.so
cp $L gpurun_out/lib_default.so.bak
for V in ${VARIANTS:-base scan4 scan512 scan256s4 apply8 emit5 grid2k grid512 base}; do
  cp dmclock_amd/variants/$V.so $L
  timeout -k 10 240 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/var_$V.json 2> gpurun_out/var_$V.err
  rc=$?; [ $rc -eq 0 ] || { echo "variant $V failed $rc"; tail -20 gpurun_out/var_$V.err; cp gpurun_out/lib_default.so.bak $L; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/var_$V.json')); print('$V', d['ms_per_step'], round(d['value']/1e6,1), {k: v for k, v in d['stages_ms_per_step'].items()})"
done
cp gpurun_out/lib_default.so.bak $L
