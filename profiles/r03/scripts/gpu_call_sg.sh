#!/bin/bash
# scalar-cache records for steps whose 64 pixels share one lattice cell and
# tetrahedron (H2S_SGATHER) A/B: C2 (hable), C4 (mobius), C3 (libplacebo)
# on smooth / uniform / website content, outputs diffed against the base
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_sg
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable mobius bt.2390; do
  KINDS=smooth,uniform,website TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_sg.so" \
    "$V/libh2s_base.so" "$V/libh2s_sg.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
