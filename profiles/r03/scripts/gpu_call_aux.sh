#!/bin/bash
# frame-load cache policy A/B (H2S_LD_AUX): nt (base), sc1 nt, sc0 sc1 nt, sc0 nt
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_aux
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable; do
  TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_a18.so" "$V/libh2s_a19.so" \
    "$V/libh2s_a3.so" "$V/libh2s_base.so" "$V/libh2s_a18.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
