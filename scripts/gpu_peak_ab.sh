#!/bin/bash
# peak-statistics A/B (scripts/bench_peak_stats.py) with a rocprofv3 kernel
# trace (CSV) beside it.  Usage: scripts/gpu_peak_ab.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-peak_ab}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/bench_peak_stats.py > "$OUT/ab.log" 2>&1 || { tail -20 "$OUT/ab.log"; exit 1; }
tail -1 "$OUT/ab.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 -u scripts/bench_peak_stats.py \
  > "$OUT/ab_prof.log" 2>&1 || { tail -20 "$OUT/ab_prof.log"; exit 1; }
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cut -c1-180 "$f" | head -12
