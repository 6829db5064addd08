#!/bin/bash
# 16-bit planar lattice (H2S_LUT16) A/B against the committed kernel: C2
# (hable) and C4 (mobius) timing with output diffs vs the base variant, then
# the full-size BASELINE configs vs the oracle on the variant
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_l16
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable mobius; do
  TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_l16.so" \
    "$V/libh2s_base.so" "$V/libh2s_l16.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_LIB=$ROOT/$V/libh2s_l16.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_00_gpu_baseline.py -k "full_size" > "$OUT/pytest_l16.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_l16.log"
exit $rc
