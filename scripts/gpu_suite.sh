#!/bin/bash
# One GPU call: the -m gpu suite (float-stage report to $OUT/float_report.jsonl),
# then the default bench line.  Each GPU step under its own limit; stop at the
# first failure.  Usage: scripts/gpu_suite.sh TAG [pytest-args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-run}; shift || true
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export H2S_FLOAT_REPORT=$OUT/float_report.jsonl
export H2S_PARITY_REPORT=$OUT/parity_report.jsonl   # exact / one-step / beyond shares per integer check
# (H2S_FLOOR_ONLY_MAX, when set, overrides the per-kind floor-only bounds)
rm -f "$H2S_FLOAT_REPORT" "$H2S_PARITY_REPORT"
timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_STOP:--x} -q --timeout 300 --timeout-method thread "$@" \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log"
