#!/bin/bash
# build the engine at git HEAD (dmclock_amd/variants/head.so) and the working
# tree (variants/cur.so) for an A/B run on one box (scripts/gpu_ab_run.sh)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/a/b/csrc $T/a/include $R/dmclock_amd/variants
for f in $(git -C $R ls-tree --name-only HEAD dmclock_amd/csrc/ | xargs -n1 basename); do
  git -C $R show HEAD:dmclock_amd/csrc/$f > $T/a/b/csrc/$f
done
git -C $R show HEAD:include/dmclock_gpu.h > $T/a/include/dmclock_gpu.h
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
/opt/rocm/bin/hipcc $F -o $R/dmclock_amd/variants/head.so $T/a/b/csrc/dmc_engine.hip &
/opt/rocm/bin/hipcc $F -o $R/dmclock_amd/variants/cur.so $R/dmclock_amd/csrc/dmc_engine.hip &
wait
rm -rf $T
