#!/bin/bash
# Round-5 check of one change: the -m gpu suite, smoke() and the bench line.
# Usage: scripts/gpu_r05_quick.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-quick}
OUT=$ROOT/gpurun_out/$TAG
cd "$ROOT"
bash scripts/gpu_r05.sh "$TAG" || exit $?
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
cut -c1-300 "$OUT/bench.json"
