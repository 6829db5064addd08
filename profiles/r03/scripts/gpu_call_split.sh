#!/bin/bash
# fast body + per-chain schedulers (CPU chain: max-memory-clause; libplacebo
# branch: default) against the committed build, C2 and C3; then the full suite
# and bench on the in-tree build
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_split
mkdir -p "$OUT"
cd "$ROOT"
V=scripts/variants
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 300 python -u scripts/time_variants.py "$V/libh2s_base.so" "$V/libh2s_split.so" \
    "$V/libh2s_base.so" "$V/libh2s_split.so" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
rm -f $V/*.so
exec_suite() { bash scripts/gpu_suite.sh r03_split_suite; }
exec_suite
