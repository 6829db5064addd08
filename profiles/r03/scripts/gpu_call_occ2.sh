#!/bin/bash
# occupancy / tiles-per-block re-check after the scalar-record steps (less
# vector-memory pressure may move the optimum): 5 (HEAD), 6 and 4 waves per
# SIMD; 4, 8 and 16 tiles per block
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_occ2
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
KINDS=smooth,uniform,website TM=hable timeout -k 10 500 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_w6.so" \
  "$V/libh2s_w4.so" "$V/libh2s_base.so@H2S_TILES_PER_BLOCK=4" "$V/libh2s_base.so@H2S_TILES_PER_BLOCK=16" "$V/libh2s_base.so" \
  "$V/libh2s_w6.so" > "$OUT/time_hable.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_hable.log"; exit 1; }
cat "$OUT/time_hable.log"
