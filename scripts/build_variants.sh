#!/bin/bash
# Launch-shape variants of the engine (same results, different launch
# parameters) for scripts/gpu_variants.sh: dmclock_amd/variants/<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/dmclock_amd/variants
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -Wno-unused-function"
SRC=$R/dmclock_amd/csrc/dmc_engine.hip
build() { /opt/rocm/bin/hipcc $FLAGS "${@:2}" -o $OUT/$1.so $SRC & }
build base
build scan4 -DDMC_SCAN_SLOTS=4
build scan512 -DDMC_SCAN_BLOCK=512
build scan256s4 -DDMC_SCAN_BLOCK=256 -DDMC_SCAN_SLOTS=4
build apply8 -DDMC_APPLY_MINB=8
build emit5 -DDMC_EMIT_MINB=5
build grid2k -DDMC_WALK_GRID_CAP=2048
build grid512 -DDMC_WALK_GRID_CAP=512
wait
ls -la $OUT
