#!/bin/bash
# One pytest selection ($PYTEST_K) run once per variant in $VARIANTS
# (dmclock_amd/variants/<name>.so through DMC_LIB): which build fails it.
# Every variant runs (a failing one is reported, not fatal); a timeout or a
# crash ends the call.
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out
for v in $VARIANTS; do
  DMC_LIB=$R/dmclock_amd/variants/$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
      -p no:cacheprovider --timeout 240 --timeout-method thread -k "$PYTEST_K" \
      > gpurun_out/iso_$v.log 2>&1
  rc=$?
  echo "$v exit $rc: $(tail -1 gpurun_out/iso_$v.log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
