#!/bin/bash
# the float-stage checks on both kernels with the report
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/r03_float
mkdir -p "$OUT"
cd "$ROOT"
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
rm -f "$H2S_FLOAT_REPORT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu --maxfail=30 \
  tests/test_00_gpu_baseline.py tests/test_gpu_parity.py -k "float" > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
exit $rc
