#!/bin/bash
# branch-free tile body (no exact-path ballot on tiles of legal codes) A/B,
# C2 and C3, then parity on the variant
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_fb
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_fb.so" "$V/libh2s_fbdef.so" \
    "$V/libh2s_base.so" "$V/libh2s_fb.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_LIB=$ROOT/$V/libh2s_fb.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_switches.py > "$OUT/pytest_fb.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_fb.log"
exit $rc
