#!/bin/bash
# Launch-shape / layout variants of the engine (same results) for A/B runs
# loaded through DMC_LIB (scripts/gpu_variants.sh): dmclock_amd/variants/<name>.so
#   usage: scripts/build_variants.sh name:-DFLAG=1,-DOTHER=2 name2:...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/dmclock_amd/variants
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
SRC=$R/dmclock_amd/csrc/dmc_engine.hip
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}; [ "$defs" = "$spec" ] && defs=""
  /opt/rocm/bin/hipcc $FLAGS ${defs//,/ } -o $OUT/$name.so $SRC &
done
wait
ls -la $OUT
