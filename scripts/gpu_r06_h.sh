#!/bin/bash
# Round 6: C2 with the lattice lookup software-pipelined one step ahead
# (profiles/r06/ab_patches/c2_pipelined.patch) at 4 and 5 waves per SIMD, and
# the product at 4 waves, against the product; same box, two rounds, output
# diffed against the first library.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_h}
mkdir -p "$OUT"
cd "$ROOT"
P=hdr-to-sdr_amd/hdr2sdr/libh2s.so
V=scripts/variants
rm -f /tmp/ref_hable_*.npy
KINDS=smooth,website,uniform timeout -k 10 600 python -u scripts/time_variants.py $P $V/libh2s_pipe4.so $V/libh2s_pipe5.so \
  $V/libh2s_wpe4.so $P $V/libh2s_pipe4.so $V/libh2s_pipe5.so $V/libh2s_wpe4.so > "$OUT/c2_pipe.log" 2>&1 ||
  { tail -5 "$OUT/c2_pipe.log"; exit 1; }
cat "$OUT/c2_pipe.log"
