#!/bin/bash
# A/B/... on one box: the variants named in $VARIANTS (dmclock_amd/variants/
# <name>.so, scripts/build_variants.sh), alternating, $ROUNDS rounds, each a
# bench.py run (stage-timed pass included) loaded through DMC_LIB.
# A variant whose run dispatches a different number of decisions than the
# first variant's (the base) is a wrong-result build, not a timing: the
# script stops with an error instead of reporting its time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
base=""
for round in $(seq ${ROUNDS:-2}); do
for v in $VARIANTS; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 240 python bench.py --no-cpu-baseline --steps 20 ${BENCH_ARGS} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { tail -5 gpurun_out/var_$v.err; exit 1; }
  dec=$(python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); c=d.get('engine_counters') or {}; print(c.get('decisions', d.get('tracker_known_frac')), c.get('bad_rounds'))") || exit 1
  [ -z "$base" ] && base="$dec"
  if [ "$dec" != "$base" ]; then
    echo "variant $v: decisions/bad_rounds $dec differ from the base's $base: wrong result, not timed"
    exit 1
  fi
  python -c "import json; d=json.load(open('gpurun_out/var_$v.json')); c=d.get('engine_counters') or {}; print('$v', d['ms_per_step'], {k: round(v*1e3,1) for k, v in (d.get('stages_ms_per_step') or {}).items()}, 'dec', c.get('decisions'), 'retries', c.get('sample_retries'))"
done
done
