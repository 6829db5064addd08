#!/bin/bash
# quad sums by ds_swizzle + full-rate adds vs DPP adds: timing on C2 / C3,
# then the tile parity tests on the variant
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_swz
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_swz.so" "$V/libh2s_base.so" "$V/libh2s_swz.so" \
    > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_LIB=$ROOT/$V/libh2s_swz.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_00_gpu_baseline.py tests/test_gpu_parity.py > "$OUT/pytest_swz.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_swz.log"
exit $rc
