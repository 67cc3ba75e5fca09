#!/bin/bash
# build the engine as it was at a git commit, for A/B runs on one box
# (scripts/gpu_variants.sh loads dmclock_amd/variants/<name>.so via DMC_LIB)
#   usage: scripts/build_at.sh <commit> <name> [-DFLAG=1 ...]
#   (<commit> "." = the working tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
c=$1; name=$2; shift 2
mkdir -p $R/dmclock_amd/variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
if [ "$c" = "." ]; then
  exec /opt/rocm/bin/hipcc $F "$@" -o $R/dmclock_amd/variants/$name.so $R/dmclock_amd/csrc/dmc_engine.hip
fi
T=$(mktemp -d)
mkdir -p $T/a/b/csrc $T/a/include
for f in $(git -C $R ls-tree --name-only $c dmclock_amd/csrc/ | xargs -n1 basename); do
  git -C $R show $c:dmclock_amd/csrc/$f > $T/a/b/csrc/$f
done
git -C $R show $c:include/dmclock_gpu.h > $T/a/include/dmclock_gpu.h
/opt/rocm/bin/hipcc $F "$@" -o $R/dmclock_amd/variants/$name.so $T/a/b/csrc/dmc_engine.hip
rm -rf $T
