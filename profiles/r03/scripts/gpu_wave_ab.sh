#!/bin/bash
# k_tile vs k_wave: timing + bit-exact output comparison (time_variants), then
# the parity suite on k_wave.  Each GPU step under its own limit.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-wave_ab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
LIB=hdr-to-sdr_amd/hdr2sdr/libh2s.so
for tmn in hable bt.2390; do
  TM=$tmn timeout -k 10 300 python -u scripts/time_variants.py "$LIB@H2S_KERNEL=tile" "$LIB@H2S_KERNEL=wave" \
    "$LIB@H2S_KERNEL=tile" "$LIB@H2S_KERNEL=wave" > "$OUT/time_$tmn.log" 2>&1 || { echo "timing $tmn failed"; cat "$OUT/time_$tmn.log"; exit 1; }
  cat "$OUT/time_$tmn.log"
done
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
H2S_KERNEL=wave timeout -k 10 600 python -u -m pytest tests/test_00_gpu_baseline.py tests/test_gpu_parity.py \
  tests/test_gpu_switches.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_wave.log" 2>&1
rc=$?
tail -5 "$OUT/pytest_wave.log"
exit $rc
