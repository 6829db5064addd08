#!/bin/bash
# Frame I/O cache-policy variants of the tile kernels (scripts/build_ablation.sh
# NAME none "-DH2S_NT_LOAD=.. -DH2S_NT_STORE=.."): the libplacebo branch's
# timings (its table lives in the L2) and C2's, product alternating, two rounds.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_n}
VARS=${2:-}
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2; do
  for v in product $VARS; do
    lib=""; [ $v != product ] && lib=$ROOT/scripts/variants/libh2s_$v.so
    H2S_LIB=$lib timeout -k 10 200 python -u scripts/time_lp_variants_r06.py ${v}_$i >> "$OUT/lp_time.log" 2>&1 ||
      { echo "$v failed"; tail -5 "$OUT/lp_time.log"; exit 1; }
  done
done
grep '^{' "$OUT/lp_time.log" | cut -c1-400
libs="$ROOT/hdr-to-sdr_amd/hdr2sdr/libh2s.so"
for v in $VARS; do libs="$libs $ROOT/scripts/variants/libh2s_$v.so"; done
KINDS=smooth,uniform,website timeout -k 10 600 python -u scripts/time_variants.py $libs > "$OUT/c2_time.log" 2>&1 || { tail -5 "$OUT/c2_time.log"; exit 1; }
tail -12 "$OUT/c2_time.log" | cut -c1-300
