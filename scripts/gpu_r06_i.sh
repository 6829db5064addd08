#!/bin/bash
# Round 6: the libplacebo instances' table locality -- a block's 8 tiles as a
# 4 x 2 patch (profiles/r06/ab_patches/patch_walk_r06.patch) and 4 / 16 tiles
# per block -- against the product, same box, two rounds.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_i}
mkdir -p "$OUT"
cd "$ROOT"
P=$ROOT/hdr-to-sdr_amd/hdr2sdr/libh2s.so
W=$ROOT/scripts/variants/libh2s_pwalk.so
for i in 1 2; do
  for v in product pwalk tpb4 tpb16; do
    lib=$P; extra=""
    [ $v = pwalk ] && lib=$W
    [ $v = tpb4 ] && extra="H2S_TILES_PER_BLOCK=4"
    [ $v = tpb16 ] && extra="H2S_TILES_PER_BLOCK=16"
    timeout -k 10 200 env H2S_LIB=$lib $extra python -u scripts/time_lp_variants_r06.py ${v}_$i >> "$OUT/lp_walk.log" 2>&1 ||
      { echo "$v failed"; tail -5 "$OUT/lp_walk.log"; exit 1; }
  done
done
grep '^{' "$OUT/lp_walk.log"
