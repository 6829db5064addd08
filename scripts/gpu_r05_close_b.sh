#!/bin/bash
# Round-5 closing run, part B at the final tree: the tests added after part A,
# the C2 / C3 profiles (scripts/gpu_r05_prof.sh) and the default bench line
# again (bench.py's side configurations now average 20 calls).
# Usage: scripts/gpu_r05_close_b.sh TAG
set -u -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-closing2}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "lut_sizes" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_b.log" 2>&1 || { tail -5 "$OUT/pytest_b.log"; exit 1; }
tail -1 "$OUT/pytest_b.log"
bash scripts/gpu_r05_prof.sh "$TAG" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
grep -E "traffic.json" "$OUT/prof.log" | cut -c1-200
timeout -k 10 400 python -u bench.py > "$OUT/bench_b.log" 2>&1 || { echo "bench failed"; tail -5 "$OUT/bench_b.log"; exit 1; }
tail -1 "$OUT/bench_b.log" > "$OUT/bench_b.json"
cut -c1-300 "$OUT/bench_b.json"
