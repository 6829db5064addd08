#!/bin/bash
# 8-byte Y'CbCr records gathered as r-pairs (H2S_PAIR8: 3 16-byte gathers per
# lookup instead of 4 12-byte ones) A/B, then parity of the variant's product
# path (its debug instances are the base build's, so the float checks are skipped)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_p8
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable mobius; do
  KINDS=smooth,uniform,website TM=$tmn timeout -k 10 500 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_p8.so" \
    "$V/libh2s_base.so" "$V/libh2s_p8.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_LIB=$ROOT/$V/libh2s_p8.so timeout -k 10 600 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py \
  tests/test_gpu_switch_matrix.py -m gpu -q --timeout 120 --timeout-method thread -k "not float" > "$OUT/pytest_p8.log" 2>&1
rc=$?
grep -E "FAILED|passed|failed" "$OUT/pytest_p8.log" | tail -8
exit $rc
