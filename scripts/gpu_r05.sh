#!/bin/bash
# Round-5 GPU call: the -m gpu suite (up to 40 failures reported, parity and
# float reports beside it), then optional diagnostics, each under its own
# limit; stop at the first failing step.  Usage: scripts/gpu_r05.sh TAG [diag...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
export H2S_PARITY_REPORT=$OUT/parity_report.jsonl
rm -f "$H2S_FLOAT_REPORT" "$H2S_PARITY_REPORT"
if [ "${SKIP_SUITE:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=60 -q --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -5 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for d in "$@"; do
  echo "=== $d"
  timeout -k 10 300 python -u $d > "$OUT/$(basename $d .py).log" 2>&1 || { echo "$d failed"; tail -5 "$OUT/$(basename $d .py).log"; exit 1; }
  tail -4 "$OUT/$(basename $d .py).log"
done
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
  tail -1 "$OUT/bench.log" | cut -c1-600
fi
