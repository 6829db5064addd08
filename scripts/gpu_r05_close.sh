#!/bin/bash
# Round-5 closing run at the final tree, part A: the -m gpu suite (with the
# parity and float reports), smoke(), the C3 diagnostics and the default bench
# line.  Part B is scripts/profile.sh for C2 and C3.  Outputs under
# gpurun_out/TAG/.  Usage: scripts/gpu_r05_close.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-closing}
OUT=$ROOT/gpurun_out/$TAG
cd "$ROOT"
bash scripts/gpu_r05.sh "$TAG" tests/diag/diag_c3_kernels.py || exit $?
echo "=== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > "$OUT/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "=== bench"
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
cut -c1-300 "$OUT/bench.json"
