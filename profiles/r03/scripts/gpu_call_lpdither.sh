#!/bin/bash
# the libplacebo branch with the S6 swscale dither: HEAD's library (expected to
# fail: its tile kernel added the luma dither offset to lut3d's R), then the fix
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_lpdither
mkdir -p "$OUT"
cd "$ROOT"
H2S_LIB=$ROOT/scripts/variants/libh2s_head.so timeout -k 10 300 python -u -m pytest tests/test_gpu_switches.py -m gpu -q \
  --timeout 120 --timeout-method thread -k "sws_dither" > "$OUT/head.log" 2>&1
echo "head rc=$?"; tail -4 "$OUT/head.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/fixed_suite.log" 2>&1
rc=$?
tail -3 "$OUT/fixed_suite.log"
exit $rc
