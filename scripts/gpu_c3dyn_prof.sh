#!/bin/bash
# C3 under peak_detect=1: the peak tests, then a rocprofv3 kernel trace of the
# bench's C3_dyn form (16 4K frames per call), stats + kernel-trace CSV under
# gpurun_out/TAG/.  Usage: scripts/gpu_c3dyn_prof.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-c3dyn}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py tests/test_00_gpu_baseline.py -m gpu -q --timeout 120 \
  --timeout-method thread -k "peak or sequence" > "$OUT/pytest_peak.log" 2>&1 || { tail -20 "$OUT/pytest_peak.log"; exit 1; }
tail -2 "$OUT/pytest_peak.log"
ARGS="--steps 40 --warmup 5 --frames 16 --tonemapper bt.2390 --gamma 1.0 --pipeline libplacebo --no-alt --no-sharded --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dyn" -o run -- python3 -u bench.py $ARGS --peak-detect \
  > "$OUT/bench_dyn.log" 2>&1 || { tail -20 "$OUT/bench_dyn.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_static" -o run -- python3 -u bench.py $ARGS \
  > "$OUT/bench_static.log" 2>&1 || { tail -20 "$OUT/bench_static.log"; exit 1; }
for d in prof_dyn prof_static; do
  f=$(find "$OUT/$d" -name '*kernel_stats.csv' | head -1)
  echo "== $d"; cut -c1-160 "$f" | head -8
done
