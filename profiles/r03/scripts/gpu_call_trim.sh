#!/bin/bash
# VALU trims now that the VALU is the busier unit (after the scalar-record
# steps): corner selects by equality with max / min (H2S_SEL_EQ) and a
# two-register uniformity key (H2S_KEY2), C2 and C4
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_trim
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable mobius; do
  KINDS=smooth,uniform,website TM=$tmn timeout -k 10 500 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_seleq.so" \
    "$V/libh2s_key2.so" "$V/libh2s_both.so" "$V/libh2s_base.so" "$V/libh2s_both.so" > "$OUT/time_$tmn.log" 2>&1 \
    || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
