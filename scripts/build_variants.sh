#!/bin/bash
# Build libh2s variants for scripts/time_variants.py.
# Usage: bash scripts/build_variants.sh NAME:"-DFLAG ..." NAME2:"..."
# Outputs scripts/variants/libh2s_NAME.so (git-ignored, travels with gpurun).
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
C=$ROOT/hdr-to-sdr_amd/csrc
mkdir -p "$ROOT/scripts/variants"
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -shared -fPIC \
    -Wno-unused-value -Wno-unused-result $flags -o "$ROOT/scripts/variants/libh2s_$name.so" \
    "$C/h2s_api.hip" "$C/h2s_kernels.hip" "$C/h2s_fast.hip" "$C/h2s_preview.hip" "$C/h2s_cube.cpp" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
ls -la "$ROOT/scripts/variants"
