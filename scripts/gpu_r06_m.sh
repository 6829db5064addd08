#!/bin/bash
# The libplacebo branch with the lut3d table as 3-byte entries
# (profiles/r06/ab_patches/lut8x_3byte.patch, scripts/build_ablation.sh):
# output checksums of product and variant, then timings alternating, two rounds.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_m}
V=${2:-lut8x_3byte}
mkdir -p "$OUT"
cd "$ROOT"
for v in product $V; do
  lib=""; [ $v != product ] && lib=$ROOT/scripts/variants/libh2s_$v.so
  H2S_LIB=$lib timeout -k 10 300 python -u scripts/lp_output_checksum.py $v >> "$OUT/checksum.log" 2>&1 || { echo "$v checksum failed"; tail -5 "$OUT/checksum.log"; exit 1; }
done
grep '^{' "$OUT/checksum.log"
for i in 1 2; do
  for v in product $V; do
    lib=""; [ $v != product ] && lib=$ROOT/scripts/variants/libh2s_$v.so
    H2S_LIB=$lib timeout -k 10 200 python -u scripts/time_lp_variants_r06.py ${v}_$i >> "$OUT/lp_time.log" 2>&1 ||
      { echo "$v failed"; tail -5 "$OUT/lp_time.log"; exit 1; }
  done
done
grep '^{' "$OUT/lp_time.log"
