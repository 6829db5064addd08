#!/bin/bash
# k_tile with the fast body: 4 waves per SIMD (98 VGPRs) and 4 / 16 tiles per
# block against the product build (5 waves, 8 tiles), C2 and C3
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_wpe
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 300 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_wpe4.so" \
    "$V/libh2s_base.so@H2S_TILES_PER_BLOCK=4" "$V/libh2s_base.so@H2S_TILES_PER_BLOCK=16" \
    "$V/libh2s_base.so" "$V/libh2s_wpe4.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
