#!/bin/bash
# Round-6 peak statistics A/B: the peak-detect GPU tests, then
# scripts/bench_peak_stats.py plain and under a rocprofv3 kernel trace
# (per-kernel durations of the quad form vs round 5's row form).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-r06_peak}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_peak_detect.py tests/test_gpu_io_matrix.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python -u scripts/bench_peak_stats.py > "$OUT/bench_peak.log" 2>&1 || { tail -5 "$OUT/bench_peak.log"; exit 1; }
tail -1 "$OUT/bench_peak.log"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 scripts/bench_peak_stats.py \
  > "$OUT/trace.log" 2>&1 || { tail -5 "$OUT/trace.log"; exit 1; }
find "$OUT/trace" -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-220 | head -20
python3 scripts/trace_by_grid.py $(find "$OUT/trace" -name "*kernel_trace.csv" | head -1) peak
