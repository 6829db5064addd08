#!/bin/bash
# A/B of k_tile variants (HEAD build, trims, trims + frame I/O issued in
# step 7) on C2 hable and C3 bt.2390, then the tile parity tests on both new
# variants
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_late
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 300 python -u scripts/time_variants.py "$V/libh2s_head.so" "$V/libh2s_late0.so" "$V/libh2s_late1.so" \
    "$V/libh2s_head.so" "$V/libh2s_late1.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
for v in late1 late0; do
  H2S_LIB=$ROOT/$V/libh2s_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_switches.py tests/test_peak_detect.py > "$OUT/pytest_$v.log" 2>&1
  rc=$?
  tail -3 "$OUT/pytest_$v.log"
  [ $rc -eq 0 ] || exit $rc
done
