#!/bin/bash
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_w6
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
TM=hable timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_w6.so" "$V/libh2s_base.so" "$V/libh2s_w6.so" \
  > "$OUT/time_hable.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_hable.log"; exit 1; }
cat "$OUT/time_hable.log"
