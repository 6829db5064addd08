#!/bin/bash
# Round 6: the libplacebo steps' table reads with 1 (product), 2 or 3 steps
# in flight (profiles/r06/ab_patches/lp_pipe_depth*.patch), same box, two
# rounds; then the libplacebo GPU tests on the product.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_j}
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2; do
  for v in product pd2 pd3; do
    lib=$ROOT/hdr-to-sdr_amd/hdr2sdr/libh2s.so
    [ $v != product ] && lib=$ROOT/scripts/variants/libh2s_$v.so
    timeout -k 10 200 env H2S_LIB=$lib python -u scripts/time_lp_variants_r06.py ${v}_$i >> "$OUT/lp_depth.log" 2>&1 ||
      { echo "$v failed"; tail -5 "$OUT/lp_depth.log"; exit 1; }
  done
done
grep '^{' "$OUT/lp_depth.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -k "libplacebo or lp_ or c3 or lut8x or peak or website" > "$OUT/pytest_lp.log" 2>&1
rc=$?
tail -2 "$OUT/pytest_lp.log"
exit $rc
