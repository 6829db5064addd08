#!/bin/bash
# CU-interleaved persistent walk (H2S_CU_WALK=1) A/B against the
# block-per-tile-run grid on one library: C2 (hable), C4 (mobius), C3 (the
# libplacebo branch) timing with output diffs, then the GPU suite with the walk on
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_cuwalk
mkdir -p "$OUT"
cd "$ROOT"
L=hdr-to-sdr_amd/hdr2sdr/libh2s.so
for tmn in hable mobius bt.2390; do
  TM=$tmn timeout -k 10 400 python -u scripts/time_variants.py "$L@H2S_CU_WALK=0" "$L@H2S_CU_WALK=1" \
    "$L@H2S_CU_WALK=0" "$L@H2S_CU_WALK=1" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
H2S_CU_WALK=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
exit $rc
