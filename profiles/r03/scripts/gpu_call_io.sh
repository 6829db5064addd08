#!/bin/bash
# I/O-wave A/B: timing of the tile-kernel variants, then the tile parity tests
# on the first variant library
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_io
mkdir -p "$OUT"
cd "$ROOT"
LIB=hdr-to-sdr_amd/hdr2sdr/libh2s.so
V=scripts/variants
for tmn in hable; do
  TM=$tmn timeout -k 10 300 python -u scripts/time_variants.py "$LIB" "$V/libh2s_iow5.so" "$V/libh2s_iow7.so" "$LIB" \
    > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_LIB=$ROOT/$V/libh2s_iow5.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_00_gpu_baseline.py tests/test_gpu_parity.py tests/test_gpu_switches.py > "$OUT/pytest_iow5.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_iow5.log"
exit $rc
